#!/bin/bash
# Top-k / threshold per-kernel times (cold cache), codec bench JSON.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/codec}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py > $O/kern.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_codec -o codec -- python3 bench/codec_bench.py --sizes 25557032 --specs int8,topk:0.01,threshold:0.02:0.05 --no-host > $O/prof_codec.log 2>&1 &&
timeout -k 10 200 python -u bench/codec_bench.py --sizes 1000000,25557032 --specs bf16,int8,topk:0.01,topk_int8:0.01,threshold:0.02:0.05 --no-host --out $O/codec_bench.json > $O/codec.log 2>&1
rc=$?
tail -n 3 $O/*.log
exit $rc
