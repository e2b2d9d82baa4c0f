#!/bin/bash
# host-side cProfile of the N=1 bench: which Python calls block (host waits on the GPU / PS)
set -o pipefail
mkdir -p gpurun_out/hostprof
timeout -k 10 300 python -m cProfile -o gpurun_out/hostprof/bench.prof bench.py --steps 20 --warmup 8 > gpurun_out/hostprof/bench.log 2>&1 || { tail -20 gpurun_out/hostprof/bench.log; exit 1; }
python - <<'PY' > gpurun_out/hostprof/top.txt
import pstats
p = pstats.Stats("gpurun_out/hostprof/bench.prof")
p.sort_stats("tottime").print_stats(40)
p.sort_stats("cumulative").print_stats(60)
PY
head -80 gpurun_out/hostprof/top.txt
