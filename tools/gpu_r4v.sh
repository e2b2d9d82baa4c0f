#!/bin/bash
# round-4: mailbox mapping time vs size (the BERT N=2 rehearsal hung in hipIpcOpenMemHandle of an
# 8 GB mailbox, r4u) -- 2 and 4 ranks on one GPU; one size per launch, each under its own limit
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
p=29630
probe() { n=$1; mb=$2; p=$((p+1))
  timeout -k 10 100 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $p tools/ipc_probe.py $mb > $O/ipc_n${n}_${mb}.log 2>&1
  rc=$?; echo "n=$n ${mb}MB rc=$rc: $(grep mailbox $O/ipc_n${n}_${mb}.log)"
}
probe 2 64; probe 2 512; probe 2 2048; probe 4 1024; probe 2 4096; probe 2 8192
