#!/bin/bash
# conv/pool tests, full GPU suite, then N=1 bench A/B over "name:ENV=VAL ..." configs in $AB
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
if [ -n "$FULL" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
fi
IFS=';' read -ra CFGS <<< "$AB"
for cfg in "${CFGS[@]}"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_$name.json > gpurun_out/bench_$name.log 2>&1 || { echo "bench $name failed"; tail -40 gpurun_out/bench_$name.log; exit 1; }
  echo "$name $(cut -c1-190 gpurun_out/bench_$name.json | cut -c100-190)"
done
