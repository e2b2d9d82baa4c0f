#!/bin/bash
# kernel + HIP API trace of the N=1 bench; tools/stall_probe.py explains the long GPU idle gaps
set -o pipefail
SO=${STALL_OUT:-gpurun_out/stall}
mkdir -p $SO
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/hstall_$$ -o bench -- python3 $ROOT/bench.py --steps 10 --warmup 5 $BENCH_ARGS > $ROOT/$SO/prof.log 2>&1
rc=$?
cd $ROOT
K=$(find /tmp/hstall_$$ -name "bench_kernel_trace.csv" | head -1)
H=$(find /tmp/hstall_$$ -name "bench_hip_api_trace.csv" | head -1)
ls /tmp/hstall_$$/* | head -20
python3 tools/stall_probe.py "$K" "$H" $SO/stalls.txt || rc=1
exit $rc
