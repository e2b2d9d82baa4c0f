#!/bin/bash
# kernel + HIP API trace of the N=1 bench; tools/stall_probe.py explains the long GPU idle gaps
set -o pipefail
mkdir -p gpurun_out/stall
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/hstall -o bench -- python3 $ROOT/bench.py --steps 10 --warmup 5 > $ROOT/gpurun_out/stall/prof.log 2>&1
rc=$?
cd $ROOT
K=$(find /tmp/hstall -name "bench_kernel_trace.csv" | head -1)
H=$(find /tmp/hstall -name "bench_hip_api_trace.csv" | head -1)
ls /tmp/hstall/* | head -20
python3 tools/stall_probe.py "$K" "$H" gpurun_out/stall/stalls.txt || rc=1
exit $rc
