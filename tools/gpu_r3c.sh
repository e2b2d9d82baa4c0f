#!/bin/bash
# round-3 check: small top-k + codec sizes, gemm2 tests, async PS GPU tests (push_early on by
# default), headline bench + tuner dump, PS update latency (model vs bucket, N=1 and emulated 7)
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
T="timeout -k 10 400"
BENCH=1 bash tools/gpu_topk_small.sh || exit 1
$T python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ps_async_gpu.py > $O/ps_gpu.log 2>&1 || { tail -30 $O/ps_gpu.log; exit 1; }
tail -1 $O/ps_gpu.log
LAT=1 bash tools/gpu_emulate.sh || exit 1
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_resnet_trajectory_gpu.py > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
tail -1 $O/traj.log
