#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_fused_bn.py tests/test_kernels_gpu.py -x -q > gpurun_out/bn_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/bn_tests.log; exit 1; }
tail -1 gpurun_out/bn_tests.log
timeout -k 10 300 python tools/bench_bn.py > gpurun_out/bench_bn.log 2>&1 || { echo "bn micro failed"; tail -30 gpurun_out/bench_bn.log; exit 1; }
cat gpurun_out/bench_bn.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_fused.json > gpurun_out/bench_fused.log 2>&1 || { echo "bench fused failed"; tail -40 gpurun_out/bench_fused.log; exit 1; }
cat gpurun_out/bench_fused.json
