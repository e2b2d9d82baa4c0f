#!/bin/bash
# round-4 N>1 readiness on one GPU: the driver's N=2/4 launch (ranks share cuda:0, gloo
# rendezvous) and the emulated N=8 PS load (7 remote workers' messages on the co-located PS)
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export HIPPS_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 10 --warmup 3 --batch 64 --out $O/reh_n$n.json > $O/reh_n$n.log 2>&1 || { echo "n=$n failed"; tail -40 $O/reh_n$n.log; exit 1; }
  cut -c1-300 $O/reh_n$n.json
done
unset HIPPS_BACKEND
timeout -k 10 400 python -u bench.py --steps 30 --warmup 8 --emulate-remote 7 --out $O/emu_er7.json > $O/emu_er7.log 2>&1 || { tail -30 $O/emu_er7.log; exit 1; }
cut -c1-300 $O/emu_er7.json
