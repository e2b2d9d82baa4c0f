#!/bin/bash
# round-4: host idle tasks no longer run from the fc layer's backward -- GPU tests, the N=1
# headline twice and a steady-state kernel table
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_shadow_linear_gpu.py tests/test_bf16_shadow.py tests/test_ps_async_gpu.py tests/test_resnet_trajectory_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --out $O/bench_n1_r$r.json > $O/bench_r$r.log 2>&1 || { echo "bench failed"; tail -40 $O/bench_r$r.log; exit 1; }
  cut -c1-200 $O/bench_n1_r$r.json
done
STEPS=12 bash tools/gpu_prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
cp gpurun_out/prof/steady.txt $O/steady.txt
head -16 $O/steady.txt
