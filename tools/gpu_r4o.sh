#!/bin/bash
# round-4: Linear layers on the bf16 weight shadow (_ShadowLinear) and the fused bf16
# cross-entropy -- their GPU tests, then the transformer configs with each on / off (same box)
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_shadow_linear_gpu.py tests/test_xent_gpu.py tests/test_bf16_shadow.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
B="--model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5"
HIPPS_SHADOW_LINEAR=1 HIPPS_FUSED_XENT=1 run bert_on $B || exit 1
HIPPS_SHADOW_LINEAR=0 HIPPS_FUSED_XENT=1 run bert_sl0 $B || exit 1
HIPPS_SHADOW_LINEAR=1 HIPPS_FUSED_XENT=0 run bert_xent0 $B || exit 1
HIPPS_SHADOW_LINEAR=0 HIPPS_FUSED_XENT=0 run bert_off $B || exit 1
L="--model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 10 --warmup 3"
HIPPS_SHADOW_LINEAR=1 HIPPS_FUSED_XENT=1 run llama1b_on $L || exit 1
HIPPS_SHADOW_LINEAR=0 HIPPS_FUSED_XENT=0 run llama1b_off $L || exit 1
run llama8b_on --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2 || exit 1
