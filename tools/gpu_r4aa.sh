#!/bin/bash
# round-4: direct push (rank 0's hook-time buckets encoded straight into its mailbox ring) --
# GPU tests, same-box A/B on ResNet-50 (two interleaved rounds) and Llama-3-8B, N=2 rehearsal
set -o pipefail
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ps_async_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
for r in 1 2; do
  run r50_dp_r$r || exit 1
  HIPPS_DIRECT_PUSH=0 run r50_dp0_r$r || exit 1
done
L8="--model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2"
run llama8b_dp $L8 || exit 1
HIPPS_DIRECT_PUSH=0 run llama8b_dp0 $L8 || exit 1
export HIPPS_BACKEND=gloo
BENCH_HANG_DUMP=150 timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29660 bench.py --gpus 2 --steps 10 --warmup 3 --batch 64 --out $O/reh_n2.json > $O/reh_n2.log 2>&1 || { echo "n=2 failed"; grep -v "amdgpu.ids\|socket.cpp" $O/reh_n2.log | tail -40; }
cut -c1-250 $O/reh_n2.json
