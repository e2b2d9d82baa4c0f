#!/bin/bash
# round-4 final validation on a fresh box: the whole GPU suite, smoke(), the N=1 bench twice and a
# steady-state kernel table of the default build (copied to profiles/r4/final/ afterwards)
set -o pipefail
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --out $O/bench_n1_r$r.json > $O/bench_r$r.log 2>&1 || { echo "bench failed"; tail -40 $O/bench_r$r.log; exit 1; }
  cut -c1-200 $O/bench_n1_r$r.json
done
STEPS=12 bash tools/gpu_prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
cp gpurun_out/prof/steady.txt $O/steady.txt
head -12 $O/steady.txt
