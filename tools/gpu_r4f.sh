#!/bin/bash
# round-4 N>1 readiness on one GPU: the driver's N=2/4 launch (ranks share cuda:0, gloo
# rendezvous) and the emulated N=8 PS load (7 remote workers' messages on the co-located PS)
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk" > $O/ktests.log 2>&1 || { tail -30 $O/ktests.log; exit 1; }
tail -1 $O/ktests.log
for f in 0 1 2 3; do
  HIPPS_TOPK_SMALL=$f timeout -k 10 240 python -u bench/codec_bench.py --sizes 10,1000,10000,32768 --specs topk:0.01 --no-host --out $O/codec_small_f$f.json > $O/codec_small_f$f.log 2>&1 || { tail -20 $O/codec_small_f$f.log; exit 1; }
  python -c "import json;print('flags $f', [(r['n'], r['encode_us']) for r in json.load(open('$O/codec_small_f$f.json'))])"
done
timeout -k 10 240 python -u bench/codec_bench.py --sizes 25557032 --specs topk:0.01,threshold:0.02:0.05 --no-host --out $O/codec_large.json > $O/codec_large.log 2>&1 || { tail -20 $O/codec_large.log; exit 1; }
python -c "import json;print('large', [(r['codec'], r['encode_us']) for r in json.load(open('$O/codec_large.json'))])"
export HIPPS_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 10 --warmup 3 --batch 64 --out $O/reh_n$n.json > $O/reh_n$n.log 2>&1 || { echo "n=$n failed"; tail -40 $O/reh_n$n.log; exit 1; }
  cut -c1-300 $O/reh_n$n.json
done
unset HIPPS_BACKEND
timeout -k 10 400 python -u bench.py --steps 30 --warmup 8 --emulate-remote 7 --out $O/emu_er7.json > $O/emu_er7.log 2>&1 || { tail -30 $O/emu_er7.log; exit 1; }
cut -c1-300 $O/emu_er7.json
HIPPS_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --out $O/host_timing.json > $O/host_timing.log 2>&1 || { tail -20 $O/host_timing.log; exit 1; }
grep -i "host" $O/host_timing.log | tail -3
timeout -k 10 300 python -u tools/host_profile.py --out $O/host_profile.txt --steps 20 --warmup 5 > $O/host_profile.log 2>&1 || { tail -20 $O/host_profile.log; exit 1; }
head -60 $O/host_profile.txt
