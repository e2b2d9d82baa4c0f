#!/bin/bash
# same-box A/B of the round-3 session-2 paths: default vs each switch off, interleaved twice
set -o pipefail
O=gpurun_out/ab_r3b
mkdir -p $O
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/$name.json > $O/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $O/$name.log; return 1; }
  python3 -c "import json; r=json.load(open('$O/$name.json')); print('$name', r['value'], r['ms_per_step'])"
}
for rep in 1 2; do
  run on_$rep HIPPS_AB=1 &&
  run dual_off_$rep HIPPS_FUSED_DUAL=0 &&
  run s2tap_off_$rep HIPPS_S2TAP=0 &&
  run dgrad_s2_off_$rep HIPPS_DGRAD_S2=0 &&
  run bngrad_off_$rep HIPPS_FUSED_BNGRAD=0 || exit 1
done
