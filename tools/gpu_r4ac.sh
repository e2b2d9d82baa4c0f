#!/bin/bash
# round-4: more N>1 rehearsals of the driver's launch on one GPU (ranks share cuda:0, gloo) on the
# closing build: BERT-base N=4 and Llama-3-1B N=2 (large ring messages: the 0.5 GB embedding)
set -o pipefail
O=gpurun_out/r4ac
mkdir -p $O
export HIPPS_BACKEND=gloo
reh() { name=$1; n=$2; port=$3; shift 3
  BENCH_HANG_DUMP=160 timeout -k 10 175 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n "$@" --out $O/$name.json > $O/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] && cut -c1-260 $O/$name.json || grep -v "amdgpu.ids\|socket.cpp" $O/$name.log | tail -30
}
reh bert_n4 4 29671 --model bert-base --batch 4 --seq 512 --bucket-mb 4 --lr 1e-3 --steps 8 --warmup 3
reh llama1b_n2 2 29672 --model llama3-1b --batch 1 --seq 1024 --param-wire bf16 --lr 1e-3 --steps 6 --warmup 2
reh r50_thr_n2 2 29673 --batch 64 --codec topk:0.01 --steps 8 --warmup 3
