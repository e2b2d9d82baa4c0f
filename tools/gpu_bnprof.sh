#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/bnprof
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bnprof -o bn -- python3 $GRAFT_REPO_ROOT/tools/bench_bn.py > $GRAFT_REPO_ROOT/gpurun_out/bnprof/bn.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; tail -20 gpurun_out/bnprof/bn.log; exit $rc
