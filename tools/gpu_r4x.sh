#!/bin/bash
# round-4: RMSNorm kernels (Llama) and the residual add in the Linear epilogue (BERT) -- GPU tests,
# Llama-1B with the fused norm / activations on and off (same box), BERT, Llama-8B
set -o pipefail
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_act_gpu.py tests/test_shadow_linear_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
L="--model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 10 --warmup 3"
run llama1b $L || exit 1
HIPPS_FUSED_ACT=0 run llama1b_act0 $L || exit 1
run bert --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5 || exit 1
run llama8b --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2 || exit 1
