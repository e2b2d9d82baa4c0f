#!/bin/bash
# full GPU suite + smoke + N=1 bench + steady-state rocprof kernel summary
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
[ -n "$NOTESTS" ] || timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
[ -n "$NOTESTS" ] || tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 8 $BENCH_ARGS --out gpurun_out/bench_n1.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
cut -c1-240 gpurun_out/bench_n1.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/hprof -o bench -- python3 $ROOT/bench.py --steps 12 --warmup 5 $BENCH_ARGS > $ROOT/gpurun_out/prof/bench_prof.log 2>&1 || { echo "prof failed"; tail -20 $ROOT/gpurun_out/prof/bench_prof.log; exit 1; }
cd $ROOT
T=$(find /tmp/hprof -name "bench_kernel_trace.csv" | head -1)
python3 tools/steady_profile.py "$T" gpurun_out/prof/steady.txt --skip 5 --title "ResNet-50 bs256 ps_async bf16 N=1 $BENCH_ARGS"
