#!/bin/bash
# round-4: biased Linear forward on the gemm2 kBias epilogue -- its GPU test, BERT-base with the
# shadow Linear on / off (same box), and a kernel table of each (rocprofv3 --kernel-trace --stats)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_shadow_linear_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
B="--model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16"
HIPPS_SHADOW_LINEAR=1 run bert_on $B --steps 15 --warmup 5 || exit 1
HIPPS_SHADOW_LINEAR=0 run bert_sl0 $B --steps 15 --warmup 5 || exit 1
HIPPS_SHADOW_LINEAR=1 run bert_on2 $B --steps 15 --warmup 5 || exit 1
prof() { name=$1; sl=$2
  cd /tmp && HIPPS_SHADOW_LINEAR=$sl timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bprof_$name -o bert -- python3 $ROOT/bench.py $B --steps 6 --warmup 3 > $ROOT/$O/prof_$name.log 2>&1 || { tail -20 $ROOT/$O/prof_$name.log; cd $ROOT; return 1; }
  cd $ROOT
  S=$(find /tmp/bprof_$name -name "bert_kernel_stats.csv" | head -1)
  cp $S $O/kernel_stats_$name.csv
  python3 - $O/kernel_stats_$name.csv > $O/top_$name.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("9 steps (3 warmup + 6); kernel ms total", round(tot / 1e6, 2), "per step", round(tot / 9e6, 2))
for r in rows[:40]:
    print(f'{float(r["TotalDurationNs"]) / 9e6:7.3f} ms/step {int(r["Calls"]) / 9:6.1f} calls/step  {r["Name"][:120]}')
PY
  head -16 $O/top_$name.txt
}
prof on 1 && prof sl0 0
