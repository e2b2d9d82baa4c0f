#!/bin/bash
# round-4: same-box A/B of the residual add in the Linear epilogue (BERT-base, two interleaved
# rounds) and a second steady-state ResNet-50 kernel table of the final build
set -o pipefail
O=gpurun_out/r4y
mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
B="--model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5"
for r in 1 2; do
  run bert_res_r$r $B || exit 1
  HIPPS_LINEAR_RESIDUAL=0 run bert_res0_r$r $B || exit 1
done
run r50 || exit 1
STEPS=12 bash tools/gpu_prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
cp gpurun_out/prof/steady.txt $O/steady.txt
head -14 $O/steady.txt
