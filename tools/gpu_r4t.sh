#!/bin/bash
# round-4: hipps LayerNorm (csrc/ln.hip) -- GPU tests, BERT-base with it on / off (same box) and
# the BERT kernel table
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_act_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
B="--model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16"
run bert $B --steps 15 --warmup 5 || exit 1
HIPPS_FUSED_ACT=0 run bert_act0 $B --steps 15 --warmup 5 || exit 1
run bert2 $B --steps 15 --warmup 5 || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bert -o k -- python3 $ROOT/bench.py $B --steps 6 --warmup 3 > $ROOT/$O/prof_bert.log 2>&1 || { tail -20 $ROOT/$O/prof_bert.log; exit 1; }
cd $ROOT
cp $(find /tmp/prof_bert -name "k_kernel_stats.csv" | head -1) $O/kernel_stats_bert.csv
python3 - $O/kernel_stats_bert.csv > $O/top_bert.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("9 steps (3 warmup + 6); kernel ms total", round(tot / 1e6, 2), "per step", round(tot / 9e6, 2))
for r in rows[:45]:
    print(f'{float(r["TotalDurationNs"]) / 9e6:7.3f} ms/step {int(r["Calls"]) / 9:6.1f} calls/step  {r["Name"][:120]}')
PY
head -30 $O/top_bert.txt
