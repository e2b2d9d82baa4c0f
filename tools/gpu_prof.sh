#!/bin/bash
# rocprofv3 kernel-trace of the N=1 bench, summarized on the box (raw trace is too big to ship)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
STEPS=${STEPS:-12}
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/hprof -o bench -- python3 $ROOT/bench.py --steps $STEPS --warmup 5 $BENCH_ARGS > $ROOT/gpurun_out/prof/bench_prof.log 2>&1
rc=$?
cd $ROOT
T=$(find /tmp/hprof -name "bench_kernel_trace.csv" | head -1)
python3 tools/steady_profile.py "$T" gpurun_out/prof/steady.txt --skip 5 --title "ResNet-50 bs256 ps_async bf16 N=1 $BENCH_ARGS" || rc=1
cp $(find /tmp/hprof -name "bench_kernel_stats.csv" | head -1) gpurun_out/prof/ 2>/dev/null
tail -3 gpurun_out/prof/bench_prof.log
exit $rc
