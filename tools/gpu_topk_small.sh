#!/bin/bash
# small-n top-k: GPU tests + codec bench at the notebook sizes (MALL flushed between calls);
# BENCH=1 also runs the N=1 headline bench
set -o pipefail
O=gpurun_out/topk
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k topk > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u bench/codec_bench.py --sizes 10,100,1000,10000,32768 --specs topk:0.01,topk_bf16:0.01,topk_int8:0.01,bf16,int8 --no-host --out $O/codec_small.json > $O/codec_small.log 2>&1 || { tail -30 $O/codec_small.log; exit 1; }
grep -v amdgpu.ids $O/codec_small.log | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['n'], r['codec'], r['encode_us'], r['decode_acc_us'])"
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm2_gpu.py > $O/g2tests.log 2>&1 || { tail -30 $O/g2tests.log; exit 1; }
  tail -1 $O/g2tests.log
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
  python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['loss_every5'])"
  timeout -k 10 300 python -u tools/tuner_dump.py --out $O/tuner.json > $O/tuner.log 2>&1 || { tail -30 $O/tuner.log; exit 1; }
  grep kxk $O/tuner.log
fi
