#!/bin/bash
# round-3 session 2: whole GPU suite without -x (list every failure), gemm2 stage probe, bench
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 400 python -u tools/gemm2_probe.py --out $O/probe.json > $O/probe.log 2>&1 || { echo "probe failed"; tail -30 $O/probe.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
cut -c1-300 $O/bench.json
