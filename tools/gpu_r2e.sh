#!/bin/bash
# Round 2: new top-k kernels (tests + cold-cache codec bench + rocprof stats/counters), trajectory test, smoke, bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_kernels_gpu.py > $O/kern.log 2>&1 &&
timeout -k 10 300 python -u bench/codec_bench.py --out $O/codec_bench.json > $O/codec.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_codec -o codec -- python3 bench/codec_bench.py --sizes 25557032 --specs bf16,int8,topk:0.01,topk_int8:0.01,threshold:0.02:0.05 > $O/prof_codec.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch -- python3 bench/codec_bench.py --sizes 25557032 --specs int8,topk:0.01 --warm > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write -- python3 bench/codec_bench.py --sizes 25557032 --specs int8,topk:0.01 --warm > $O/pmc_write.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 550 --timeout-method thread tests/test_resnet_trajectory_gpu.py > $O/traj.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --out $O/bench.json > $O/bench.log 2>&1
rc=$?
tail -n 2 $O/*.log
exit $rc
