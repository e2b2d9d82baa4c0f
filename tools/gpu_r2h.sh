#!/bin/bash
# Round 2: top-k count/scan/write: tests, cold codec bench, per-kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_rccl_gpu.py > $O/kern.log 2>&1 &&
timeout -k 10 200 python -u bench/codec_bench.py --sizes 1000000,25557032 --specs bf16,int8,topk:0.01,topk_int8:0.01,threshold:0.02:0.05 --out $O/codec_bench.json > $O/codec.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_codec -o codec -- python3 bench/codec_bench.py --sizes 25557032 --specs int8,topk:0.01,threshold:0.02:0.05 > $O/prof_codec.log 2>&1
rc=$?
tail -n 3 $O/*.log
exit $rc
