#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_gather.json > gpurun_out/bench_gather.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_gather.log; exit 1; }
cat gpurun_out/bench_gather.json
HIPPS_GRAD_GATHER=0 timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_flat.json > gpurun_out/bench_flat.log 2>&1 || { echo "bench flat failed"; tail -40 gpurun_out/bench_flat.log; exit 1; }
cat gpurun_out/bench_flat.json
