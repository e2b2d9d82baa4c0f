#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_conv1x1_gpu.py -x -q > gpurun_out/conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 300 python tools/bench_conv1x1.py > gpurun_out/bench_conv1x1.log 2>&1 || { echo "conv bench failed"; tail -30 gpurun_out/bench_conv1x1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_conv1x1.log
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_conv.json > gpurun_out/bench_conv.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench_conv.log; exit 1; }
cat gpurun_out/bench_conv.json
HIPPS_FUSED_CONV=0 timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_noconv.json > gpurun_out/bench_noconv.log 2>&1 || { echo "bench noconv failed"; tail -40 gpurun_out/bench_noconv.log; exit 1; }
cat gpurun_out/bench_noconv.json
HIPPS_CONV_WGRAD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 6 --out gpurun_out/bench_miowgrad.json > gpurun_out/bench_miowgrad.log 2>&1 || { echo "bench miopen-wgrad failed"; tail -40 gpurun_out/bench_miowgrad.log; exit 1; }
cat gpurun_out/bench_miowgrad.json
