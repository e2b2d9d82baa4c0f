#!/bin/bash
# round-4: the N=2 BERT rehearsal hung (r4s) -- reproduce small with stack dumps, then the LN /
# pull-shadow GPU tests
set -o pipefail
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ps_async_gpu.py tests/test_act_gpu.py tests/test_bf16_shadow.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export HIPPS_BACKEND=gloo
run2() { name=$1; shift
  BENCH_HANG_DUMP=100 timeout -k 10 160 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 "$@" --out $O/$name.json > $O/$name.log 2>&1
  echo "$name rc=$?"; grep -v "amdgpu.ids\|socket.cpp\|Gloo" $O/$name.log | tail -60 | cut -c1-200
}
run2 bert_tiny_n2 --model bert-tiny --batch 4 --seq 64 --bucket-mb 0.05 --lr 1e-3 --steps 6 --warmup 2
run2 bert_n2 --model bert-base --batch 4 --seq 128 --bucket-mb 4 --lr 1e-3 --steps 6 --warmup 2
