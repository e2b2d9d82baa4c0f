#!/bin/bash
# Round 2: new async transport (device doorbells + GPU-time pull), masks, trajectory test, bench.
set -o pipefail
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "masked or sgd or adam" > $O/kern.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ps_async_gpu.py > $O/async.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 590 --timeout-method thread tests/test_resnet_trajectory_gpu.py > $O/traj.log 2>&1 &&
timeout -k 10 300 python -u tools/trajectory.py --runs async_slr,async_prefetch --out $O/traj_extra.json > $O/traj_extra.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/bench.log 2>&1
rc=$?
tail -n 3 $O/*.log
exit $rc
