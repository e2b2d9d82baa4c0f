#!/bin/bash
# Secondary BASELINE configs + codec microbenchmark on one MI355X.
set -o pipefail
mkdir -p gpurun_out/cfg
[ -n "$WITH_CODEC" ] && { timeout -k 10 300 python bench/codec_bench.py --out gpurun_out/cfg/codec_bench.json > gpurun_out/cfg/codec_bench.log 2>&1 || exit 1; }

run() { name=$1; shift; timeout -k 10 420 python bench.py "$@" --out gpurun_out/cfg/$name.json > gpurun_out/cfg/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; [ -f gpurun_out/cfg/$name.json ] && cat gpurun_out/cfg/$name.json; return $rc; }
run r50_topk_int8 --codec topk_int8:0.01 --steps 15 --warmup 5 || exit 1
run r50_int8 --codec int8 --steps 15 --warmup 5 || exit 1
run r50_fp32 --codec fp32 --steps 15 --warmup 5 || exit 1
run bert_base --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --steps 15 --warmup 5 || exit 1
run llama3_1b --model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 10 --warmup 3 || exit 1
run llama3_8b --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2
exit 0
