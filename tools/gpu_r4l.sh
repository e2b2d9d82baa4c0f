#!/bin/bash
# round-4: the side-stream weight gradients without record_stream (inputs held until an event or
# the join): the wgrad / PS / fused-BN GPU tests, the allocator probe, and a bench
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fused_bn.py tests/test_ps_async_gpu.py tests/test_resnet_trajectory_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/alloc_probe.py --out $O/alloc_probe.txt --steps 40 --warmup 5 > $O/alloc_probe.log 2>&1 || { tail -20 $O/alloc_probe.log; exit 1; }
head -14 $O/alloc_probe.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --out $O/bench_r$r.json > $O/bench_r$r.log 2>&1 || { tail -20 $O/bench_r$r.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_r$r.json'));print('bench r$r', d['value'], d['ms_per_step'], d['final_loss'])"
done
HIPPS_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --out $O/host_timing.json > $O/host_timing.log 2>&1 || { tail -20 $O/host_timing.log; exit 1; }
grep "host ms\|allocator" $O/host_timing.log
