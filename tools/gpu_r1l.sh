#!/bin/bash
# 32-bit index math in the max pool kernels: shadow/conv tests, full GPU suite, smoke, bench, profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bf16_shadow.py tests/test_conv1x1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { echo "new tests failed"; tail -60 gpurun_out/new_tests.log; exit 1; }
tail -2 gpurun_out/new_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out gpurun_out/bench_n1.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench_n1.json
timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out gpurun_out/bench_n1_again.json > gpurun_out/bench_again.log 2>&1 || { echo "bench again failed"; tail -40 gpurun_out/bench_again.log; exit 1; }
cut -c1-260 gpurun_out/bench_n1_again.json
bash tools/gpu_prof.sh
