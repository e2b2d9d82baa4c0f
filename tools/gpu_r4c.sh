#!/bin/bash
# round-4 codec + secondary-config measurements on this build: codec bench
# (cold MALL) at the notebook sizes, 32K and full-bucket sizes; HBM counters of the codec
# kernels; config 3 (ResNet-50 top-k+int8, int8, fp32 wire), config 4 (BERT-base threshold), the
# transformer configs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk or codec or threshold or q8" > $O/ktests.log 2>&1 || { tail -30 $O/ktests.log; exit 1; }
tail -1 $O/ktests.log
HIPPS_TOPK_FOLD=0 timeout -k 10 240 python -u bench/codec_bench.py --sizes 1000000,25557032 --specs topk:0.01 --no-host --out $O/codec_bench_nofold.json > $O/codec_nofold.log 2>&1 || { tail -20 $O/codec_nofold.log; exit 1; }
HIPPS_Q8_ENC=0 timeout -k 10 240 python -u bench/codec_bench.py --sizes 1000000,25557032 --specs int8 --no-host --out $O/codec_bench_q8old.json > $O/codec_q8old.log 2>&1 || { tail -20 $O/codec_q8old.log; exit 1; }
HIPPS_TOPK_PF=0 timeout -k 10 240 python -u bench/codec_bench.py --sizes 1000000,25557032 --specs topk:0.01 --no-host --out $O/codec_bench_nopf.json > $O/codec_nopf.log 2>&1 || { tail -20 $O/codec_nopf.log; exit 1; }
timeout -k 10 240 python -u bench/codec_bench.py --sizes 10,100,1000,10000,32768,1000000,25557032 --specs bf16,int8,topk:0.01,topk_int8:0.01,threshold:0.02:0.05 --no-host --out $O/codec_bench.json > $O/codec.log 2>&1 || { tail -20 $O/codec.log; exit 1; }
tail -3 $O/codec.log
ARGS="bench/codec_bench.py --sizes 25557032 --specs bf16,int8,topk:0.01,threshold:0.002:0.05 --no-host --warm"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch -- python3 $ARGS > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write -- python3 $ARGS > $O/write.log 2>&1 || exit 1
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; [ -f $O/$name.json ] && cut -c1-300 $O/$name.json; return $rc; }
run r50_topk_int8 --codec topk_int8:0.01 --steps 15 --warmup 5 || exit 1
run r50_int8 --codec int8 --steps 15 --warmup 5 || exit 1
run r50_fp32 --codec fp32 --steps 15 --warmup 5 || exit 1
run bert_base_threshold_1e-3 --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec threshold:1e-3:0.05 --steps 15 --warmup 5 || exit 1
run bert_base_bf16 --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5 || exit 1
run llama3_1b --model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 10 --warmup 3 || exit 1
run llama3_8b --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2
exit 0
