#!/bin/bash
# GPU tests + smoke + bench + traced bench (HIP-event phases) + roctx marker timeline summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out gpurun_out/bench_n1.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench_n1.json
HIPPS_TRACE=1 timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out gpurun_out/bench_n1_traced.json > gpurun_out/bench_traced.log 2>&1 || { echo "traced bench failed"; tail -40 gpurun_out/bench_traced.log; exit 1; }
cat gpurun_out/bench_n1_traced.json
