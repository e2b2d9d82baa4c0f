#!/bin/bash
# stream-priority A/B (HIPPS_WGRAD_PRIO, HIPPS_COMPUTE_PRIO: both measured no gain and were removed again; profiles/r3b/ab_wgprio)
set -o pipefail
O=gpurun_out/ab_wgprio
mkdir -p $O
timeout -k 10 120 python -c "import torch; print('priority range (low, high):', torch.cuda.Stream.priority_range())" || exit 1
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/$name.json > $O/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $O/$name.log; return 1; }
  python3 -c "import json; r=json.load(open('$O/$name.json')); print('$name', r['value'], r['ms_per_step'])"
}
for rep in 1 2; do
  run p0_$rep HIPPS_AB=1 &&
  run chi_$rep HIPPS_COMPUTE_PRIO=-1 || exit 1
done
