#!/bin/bash
# Round 2: trajectory timing (fused + plain), extra async variants, bench.
set -o pipefail
O=gpurun_out/r2b
mkdir -p $O
date +%s > $O/t0
timeout -k 10 400 python -u tools/trajectory.py --runs local,async_md0,async,async_slr,async_prefetch --out $O/fused.json > $O/fused.log 2>&1 &&
date +%s > $O/t1 &&
timeout -k 10 400 python -u tools/trajectory.py --plain --out $O/plain.json > $O/plain.log 2>&1 &&
date +%s > $O/t2 &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/bench.log 2>&1
rc=$?
date +%s > $O/t3
tail -n 2 $O/*.log
exit $rc
