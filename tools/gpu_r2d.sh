#!/bin/bash
# Round 2: full GPU suite + smoke + bench (+ rocprof kernel stats of the bench).
set -o pipefail
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 500 --timeout-method thread tests -m gpu > $O/gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --out $O/bench.json > $O/bench.log 2>&1
rc=$?
tail -n 3 $O/*.log
exit $rc
