#!/bin/bash
# round-4: byte-ring mailbox + pull-written shadow + hipps LayerNorm -- GPU tests, the driver's N>1
# launch on one GPU (ResNet-50 N=2/4, BERT-base N=2), N=1 headline twice, BERT LN A/B, Llama-8B
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ps_async_gpu.py tests/test_act_gpu.py tests/test_bf16_shadow.py tests/test_shadow_linear_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
run r50_a || exit 1
HIPPS_PULL_SHADOW=0 run r50_ps0 || exit 1
run r50_b || exit 1
B="--model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5"
run bert $B || exit 1
HIPPS_FUSED_ACT=0 run bert_act0 $B || exit 1
run llama8b --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2 || exit 1
export HIPPS_BACKEND=gloo
for n in 2 4; do
  BENCH_HANG_DUMP=150 timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29640+n)) bench.py --gpus $n --steps 10 --warmup 3 --batch 64 --out $O/reh_n$n.json > $O/reh_n$n.log 2>&1 || { echo "n=$n failed"; grep -v "amdgpu.ids\|socket.cpp" $O/reh_n$n.log | tail -40; }
  cut -c1-250 $O/reh_n$n.json
done
BENCH_HANG_DUMP=150 timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29650 bench.py --gpus 2 --model bert-base --batch 8 --seq 512 --bucket-mb 4 --lr 1e-3 --steps 10 --warmup 3 --out $O/reh_bert_n2.json > $O/reh_bert_n2.log 2>&1 || { echo "bert n=2 failed"; grep -v "amdgpu.ids\|socket.cpp" $O/reh_bert_n2.log | tail -40; }
cut -c1-250 $O/reh_bert_n2.json
unset HIPPS_BACKEND
