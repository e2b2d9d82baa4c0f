#!/bin/bash
# async GPU tests (auto shadow off for conv-free models), then the secondary BASELINE configs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ps_async_gpu.py tests/test_bf16_shadow.py -x -q --timeout 120 --timeout-method thread > gpurun_out/async_tests.log 2>&1 || { echo "async tests failed"; tail -60 gpurun_out/async_tests.log; exit 1; }
tail -1 gpurun_out/async_tests.log
bash tools/gpu_configs.sh
