#!/bin/bash
# round-4: fused SwiGLU / RoPE (csrc/act.hip), parallel colsum finalize, buckets pushed in
# completion order (messages name their bucket) -- GPU tests, then BERT / Llama benches and a
# BERT + Llama-1B kernel table
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_act_gpu.py tests/test_xent_gpu.py tests/test_shadow_linear_gpu.py tests/test_ps_async_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
B="--model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16"
run bert $B --steps 15 --warmup 5 || exit 1
run bert_thr $B --codec threshold:1e-3:0.05 --steps 15 --warmup 5 || exit 1
L="--model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 10 --warmup 3"
run llama1b $L || exit 1
HIPPS_FUSED_ACT=0 run llama1b_act0 $L || exit 1
run llama8b --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2 || exit 1
prof() { name=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o k -- python3 $ROOT/bench.py "$@" > $ROOT/$O/prof_$name.log 2>&1 || { tail -20 $ROOT/$O/prof_$name.log; cd $ROOT; return 1; }
  cd $ROOT
  cp $(find /tmp/prof_$name -name "k_kernel_stats.csv" | head -1) $O/kernel_stats_$name.csv
  python3 - $O/kernel_stats_$name.csv $2 > $O/top_$name.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("9 steps (3 warmup + 6); kernel ms total", round(tot / 1e6, 2), "per step", round(tot / 9e6, 2))
for r in rows[:45]:
    print(f'{float(r["TotalDurationNs"]) / 9e6:7.3f} ms/step {int(r["Calls"]) / 9:6.1f} calls/step  {r["Name"][:120]}')
PY
  head -20 $O/top_$name.txt
}
prof bert $B --steps 6 --warmup 3 && prof llama1b --model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 6 --warmup 3
