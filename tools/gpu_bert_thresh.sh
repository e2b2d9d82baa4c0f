#!/bin/bash
# Config 4: BERT-base async PS with the variable-size threshold codec on per-layer buckets.
set -o pipefail
O=gpurun_out/cfg4
mkdir -p $O
run() { name=$1; shift; timeout -k 10 400 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; [ -f $O/$name.json ] && cut -c1-400 $O/$name.json; return $rc; }
run bert_base_threshold_1e-4 --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec threshold:1e-4:0.05 --steps 15 --warmup 5 &&
run bert_base_threshold_1e-3 --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec threshold:1e-3:0.05 --steps 15 --warmup 5 &&
run bert_base_bf16 --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5
