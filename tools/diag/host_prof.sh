# Host-side profile (cProfile) of a short bench run: where the Python side of a step spends time.
#   bash tools/diag/host_prof.sh <out-dir> <bench args...>
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/host.prof bench.py --steps 20 --warmup 5 "$@" --out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python - "$O" <<'PY' > $O/host_top.txt
import pstats, sys
s = pstats.Stats(sys.argv[1] + "/host.prof")
s.sort_stats("tottime").print_stats(45)
s.sort_stats("cumulative").print_stats(60)
PY
head -80 $O/host_top.txt | cut -c1-160
