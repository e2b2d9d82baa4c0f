#!/bin/bash
# Round 2: trajectory without MIOpen deterministic mode (timing + bitwise local==async_md0).
set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
date +%s > $O/t0
timeout -k 10 400 python -u tools/trajectory.py --runs local,async_md0,async --out $O/fused.json > $O/fused.log 2>&1 &&
date +%s > $O/t1 &&
timeout -k 10 400 python -u tools/trajectory.py --plain --out $O/plain.json > $O/plain.log 2>&1 &&
date +%s > $O/t2 &&
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_debug_gpu.py tests/test_bf16_shadow.py > $O/gpu.log 2>&1
rc=$?
date +%s > $O/t3
tail -n 2 $O/*.log
exit $rc
