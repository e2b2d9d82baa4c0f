#!/bin/bash
# fusion round: conv/pool kernel tests, full GPU suite, A/B benches of each fusion switch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for cfg in "base:" "nograd:HIPPS_FUSED_GRAD=0" "nopool:HIPPS_FUSED_POOL=0" "bf16pub:HIPPS_PARAM_WIRE=bf16"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_$name.json > gpurun_out/bench_$name.log 2>&1 || { echo "bench $name failed"; tail -40 gpurun_out/bench_$name.log; exit 1; }
  echo "$name $(cat gpurun_out/bench_$name.json)"
done
