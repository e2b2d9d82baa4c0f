#!/bin/bash
# round-4 check: PS kernels with the cross-device acquire + slot-reuse stress, then the stall probe
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_ps_async_gpu.py > gpurun_out/r4a/tests.log 2>&1 || { tail -30 gpurun_out/r4a/tests.log; exit 1; }
tail -3 gpurun_out/r4a/tests.log
bash tools/gpu_stall.sh
