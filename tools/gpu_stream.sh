#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/st
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/st/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/st/gpu_tests.log; exit 1; }
tail -1 gpurun_out/st/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/st/bench.json > gpurun_out/st/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/st/bench.log; exit 1; }
cat gpurun_out/st/bench.json
timeout -k 10 500 python bench.py --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --bucket-mb 512 --steps 6 --warmup 2 --out gpurun_out/st/llama8b.json > gpurun_out/st/llama8b.log 2>&1; echo "llama rc=$?"
cat gpurun_out/st/llama8b.json 2>/dev/null; tail -3 gpurun_out/st/llama8b.log
