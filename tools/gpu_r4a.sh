#!/bin/bash
# round-4 check: PS kernels with the cross-device acquire + slot-reuse stress, gemm2 (in-launch
# weight-gradient reduction), a bench run, then the step-boundary stall probe
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ps_async_gpu.py tests/test_gemm2_gpu.py > gpurun_out/r4a/tests.log 2>&1 || { tail -30 gpurun_out/r4a/tests.log; exit 1; }
tail -3 gpurun_out/r4a/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --out gpurun_out/r4a/bench.json > gpurun_out/r4a/bench.log 2>&1 || { tail -20 gpurun_out/r4a/bench.log; exit 1; }
cat gpurun_out/r4a/bench.json | cut -c1-400
bash tools/gpu_stall.sh
