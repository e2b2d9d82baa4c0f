#!/bin/bash
# conv-kernel tests first (new kernels), then the full GPU suite, smoke, and A/B benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python tools/bench_conv1x1.py > gpurun_out/bench_conv1x1.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/bench_conv1x1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_conv1x1.log | tail -30
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_wgrad.json > gpurun_out/bench_wgrad.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_wgrad.log; exit 1; }
cat gpurun_out/bench_wgrad.json
HIPPS_CONV_WGRAD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_miowgrad.json > gpurun_out/bench_miowgrad.log 2>&1 || { echo "bench miopen-wgrad failed"; tail -40 gpurun_out/bench_miowgrad.log; exit 1; }
cat gpurun_out/bench_miowgrad.json
