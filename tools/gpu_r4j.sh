#!/bin/bash
# round-4: which allocations does the steady-state bench still make? (tools/alloc_probe.py, with
# and without the forward-time gradient drain)
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
for v in 1 0; do
  HIPPS_HOLD_DRAIN=$v timeout -k 10 300 python -u tools/alloc_probe.py --out $O/alloc_probe_drain$v.txt --steps 40 --warmup 5 > $O/alloc_probe_drain$v.log 2>&1 || { tail -20 $O/alloc_probe_drain$v.log; exit 1; }
  echo "== drain $v"; head -30 $O/alloc_probe_drain$v.txt
done
