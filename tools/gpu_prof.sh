#!/bin/bash
# rocprofv3 kernel-trace stats of the N=1 bench (no PMC here; counters get their own run)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
find gpurun_out/prof -name "*stats*" | head
exit $rc
