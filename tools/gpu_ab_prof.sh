#!/bin/bash
# A/B kernel tables: bench with and without an env switch (usage: gpu_ab_prof.sh VAR outdir)
set -o pipefail
export TMPDIR=/tmp
VAR=$1; O=${2:-gpurun_out/abprof}
mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
for v in 1 0; do
  export $VAR=$v; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ab$v -o b -- python3 $ROOT/bench.py --steps 12 --warmup 5 > $ROOT/$O/prof$v.log 2>&1 || exit 1
  cd $ROOT
  python3 tools/steady_profile.py $(find /tmp/ab$v -name "b_kernel_trace.csv" | head -1) $O/steady$v.txt --skip 5 --title "$VAR=$v" || exit 1
done
