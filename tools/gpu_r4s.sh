#!/bin/bash
# round-4: N>1 readiness after the bucket-named message protocol -- the driver's N=2/4 launch on
# one GPU (ranks share cuda:0, gloo rendezvous) for ResNet-50 and BERT-base (a bucket without
# gradients on every rank), then the N=1 headline twice
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
export HIPPS_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 10 --warmup 3 --batch 64 --out $O/reh_n$n.json > $O/reh_n$n.log 2>&1 || { echo "n=$n failed"; tail -40 $O/reh_n$n.log; exit 1; }
  cut -c1-300 $O/reh_n$n.json
done
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --model bert-base --batch 8 --seq 512 --bucket-mb 4 --lr 1e-3 --steps 10 --warmup 3 --out $O/reh_bert_n2.json > $O/reh_bert_n2.log 2>&1 || { echo "bert n=2 failed"; tail -40 $O/reh_bert_n2.log; exit 1; }
cut -c1-300 $O/reh_bert_n2.json
unset HIPPS_BACKEND
for r in 1 2; do
  timeout -k 10 300 python bench.py --out $O/bench_n1_r$r.json > $O/bench_r$r.log 2>&1 || { echo "bench failed"; tail -40 $O/bench_r$r.log; exit 1; }
  cut -c1-200 $O/bench_n1_r$r.json
done
