#!/bin/bash
# quick GPU check: the given test files, the N=1 bench, and the steady-state kernel profile
#   TESTS="tests/test_gemm2_gpu.py tests/test_fused_bn.py" bash tools/gpu_quick.sh
set -o pipefail
O=gpurun_out/quick
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 8 $BENCH_ARGS --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -40 $O/bench.log; exit 1; }
cut -c1-200 $O/bench.json
[ -n "$NOPROF" ] || bash tools/gpu_prof.sh
