#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tun
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 200 --timeout-method thread -k wgrad > gpurun_out/tun/tests.log 2>&1 || { tail -30 gpurun_out/tun/tests.log; exit 1; }
tail -1 gpurun_out/tun/tests.log
timeout -k 10 300 python -u tools/tuner_dump.py --out gpurun_out/tun/tuner.json > gpurun_out/tun/tuner.log 2>&1 || { tail -30 gpurun_out/tun/tuner.log; exit 1; }
grep -E "^w|sum of" gpurun_out/tun/tuner.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out gpurun_out/tun/bench.json > gpurun_out/tun/bench.log 2>&1 || { tail -30 gpurun_out/tun/bench.log; exit 1; }
cut -c1-200 gpurun_out/tun/bench.json
