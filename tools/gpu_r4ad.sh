#!/bin/bash
# round-4: bounded mailbox open that falls back to the p2p transport -- PS GPU tests, then the
# one-GPU N>1 rehearsals that hung in r4ac (BERT-base N=4, Llama-3-1B N=2) and ResNet-50 N=2
set -o pipefail
O=gpurun_out/r4ad
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ps_async_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export HIPPS_BACKEND=gloo
reh() { name=$1; n=$2; port=$3; shift 3
  BENCH_HANG_DUMP=165 timeout -k 10 175 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n "$@" --out $O/$name.json > $O/$name.log 2>&1
  rc=$?; echo "$name rc=$rc $(grep -o 'fell back[^"]*' $O/$name.log | head -1)"; [ $rc -eq 0 ] && cut -c1-200 $O/$name.json || grep -v "amdgpu.ids\|socket.cpp" $O/$name.log | grep "hipps\|Error\|error" | tail -8
}
reh r50_n2 2 29681 --batch 64 --steps 8 --warmup 3
reh bert_n4 4 29682 --model bert-base --batch 4 --seq 512 --bucket-mb 4 --lr 1e-3 --steps 8 --warmup 3
reh llama1b_n2 2 29683 --model llama3-1b --batch 1 --seq 1024 --param-wire bf16 --lr 1e-3 --steps 6 --warmup 2
