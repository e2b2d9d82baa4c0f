#!/bin/bash
# round-4: last check of the final tree -- smoke() and the N=1 headline
set -o pipefail
O=gpurun_out/r4ae
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --out $O/bench_n1.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -40 $O/bench.log; exit 1; }
cut -c1-200 $O/bench_n1.json
