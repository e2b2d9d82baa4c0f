#!/bin/bash
# Rehearse the driver's N>1 bench launch on ONE GPU: N ranks share cuda:0, gloo rendezvous.
set -o pipefail
mkdir -p gpurun_out/reh
export HIPPS_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 10 --warmup 3 --batch 64 --out gpurun_out/reh/n$n.json > gpurun_out/reh/n$n.log 2>&1 || { echo "n=$n failed"; tail -40 gpurun_out/reh/n$n.log; exit 1; }
  cat gpurun_out/reh/n$n.json
done
