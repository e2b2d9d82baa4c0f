#!/bin/bash
# HBM traffic counters of the codec kernels (one counter group per rocprofv3 pass).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/counters}
mkdir -p $O
ARGS="bench/codec_bench.py --sizes 25557032 --specs bf16,int8,topk:0.01,threshold:0.002:0.05 --no-host --warm"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch -- python3 $ARGS > $O/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write -- python3 $ARGS > $O/write.log 2>&1
rc=$?
tail -n 2 $O/*.log
exit $rc
