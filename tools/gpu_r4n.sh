#!/bin/bash
# round-4: where does the BERT-base step (secondary config) spend its GPU time?  kernel stats of
# a short run (rocprofv3 --kernel-trace --stats)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=gpurun_out/r4n
mkdir -p $O
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bprof -o bert -- python3 $ROOT/bench.py --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --steps 6 --warmup 3 > $ROOT/$O/prof.log 2>&1 || { tail -20 $ROOT/$O/prof.log; exit 1; }
cd $ROOT
S=$(find /tmp/bprof -name "bert_kernel_stats.csv" | head -1)
cp $S $O/bert_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4n/bert_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("total kernel ms", round(tot / 1e6, 2))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"]) / 1e6:8.2f} ms {int(r["Calls"]):6d} calls {float(r["Percentage"]):5.1f}%  {r["Name"][:110]}')
PY
