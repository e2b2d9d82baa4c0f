#!/bin/bash
# Loss-trajectory check: hipps fused (local), plain PyTorch, ps_async N=1 (max_delay 0 and -1).
set -o pipefail
O=gpurun_out/traj
mkdir -p $O
T="timeout -k 10 240"
$T python -u tools/trajectory.py --steps 40 --batch 64 --out $O/fused_local.json > $O/fused_local.log 2>&1 &&
$T python -u tools/trajectory.py --steps 40 --batch 64 --plain --out $O/plain.json > $O/plain.log 2>&1 &&
$T python -u tools/trajectory.py --steps 40 --batch 64 --mode ps_async --max-delay 0 --out $O/async_md0.json > $O/async_md0.log 2>&1 &&
$T python -u tools/trajectory.py --steps 40 --batch 64 --mode ps_async --max-delay -1 --out $O/async_mdinf.json > $O/async_mdinf.log 2>&1 &&
$T python -u tools/trajectory.py --steps 40 --batch 64 --bf16-weights on --codec bf16 --out $O/fused_local_shadow.json > $O/fused_local_shadow.log 2>&1 &&
$T python -u bench.py --steps 30 --warmup 5 > $O/bench.log 2>&1
rc=$?
tail -n 3 $O/*.log
exit $rc
