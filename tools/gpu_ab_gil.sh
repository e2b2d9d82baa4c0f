#!/bin/bash
# GIL switch interval A/B (HIPPS_GIL_SWITCH_US; Python default 5000 us), interleaved, with host timing
set -o pipefail
O=gpurun_out/ab_gil
mkdir -p $O
run() {
  name=$1; shift
  env HIPPS_HOST_TIMING=1 "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/$name.json > $O/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $O/$name.log; return 1; }
  python3 -c "import json; r=json.load(open('$O/$name.json')); print('$name', r['value'], r['ms_per_step'], r.get('ps_staleness_mean'))"
  grep -a "host ms" $O/$name.log
}
for rep in 1 2; do
  run base_$rep HIPPS_AB=1 &&
  run sw500_$rep HIPPS_GIL_SWITCH_US=500 &&
  run sw100_$rep HIPPS_GIL_SWITCH_US=100 || exit 1
done
