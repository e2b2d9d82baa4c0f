#!/bin/bash
# async PS mailbox depth A/B (--mailbox-slots; auto = 2 x buckets = 4 for ResNet-50), interleaved, with host timing
set -o pipefail
O=gpurun_out/ab_slots
mkdir -p $O
run() {
  name=$1; shift
  HIPPS_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/$name.json "$@" > $O/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $O/$name.log; return 1; }
  python3 -c "import json; r=json.load(open('$O/$name.json')); print('$name', r['value'], r['ms_per_step'], r.get('ps_staleness_mean'))"
  grep -a "host ms" $O/$name.log
}
for rep in 1 2; do
  run auto_$rep &&
  run s8_$rep --mailbox-slots 8 &&
  run s16_$rep --mailbox-slots 16 || exit 1
done
