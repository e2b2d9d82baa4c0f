#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 300 python tools/bench_conv1x1.py > gpurun_out/bench_conv1x1.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/bench_conv1x1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_conv1x1.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if 'total' in d: print('TOTAL', d['total']); continue
    print(d['cin'],d['hw'],d['cout'],d['stride'],'wgrad mio',d['miopen_wgrad_ms'],'own',d['hipps_wgrad_ms'],'err',d['wgrad_rel_err'])"
for cfg in "own:HIPPS_CONV_WGRAD=1" "mio:HIPPS_CONV_WGRAD=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_$name.json > gpurun_out/bench_$name.log 2>&1 || { echo "bench $name failed"; tail -40 gpurun_out/bench_$name.log; exit 1; }
  echo "$name $(cut -c1-200 gpurun_out/bench_$name.json)"
done
