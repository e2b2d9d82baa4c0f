#!/bin/bash
# stem kernels: GPU tests, hipps-vs-MIOpen microbench, N=1 bench (BENCH=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1; rc=$?; tail -4 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_stem.py > gpurun_out/stem_bench.log 2>&1; rc=$?; grep -E "^(C=3|hipps)" gpurun_out/stem_bench.log; [ $rc -eq 0 ] || exit $rc
[ -n "$BENCH" ] || exit 0
timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out gpurun_out/bench_stem.json > gpurun_out/bench_stem.log 2>&1; rc=$?; cut -c1-300 gpurun_out/bench_stem.json; exit $rc
