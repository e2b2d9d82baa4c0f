# Steady-state kernel table of a transformer config at N=1 (rocprofv3 --kernel-trace --stats)
#   bash tools/diag/tf_prof.sh <out> <model> [bench args...]
set -o pipefail
O=gpurun_out/$1; M=$2; shift 2; mkdir -p $O
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tfprof -o tf -- \
  python3 "$ROOT/bench.py" --model $M --steps 8 --warmup 3 "$@") > $O/prof.log 2>&1 || exit 1
T=$(find /tmp/tfprof -name "tf_kernel_trace.csv" | head -1)
python3 tools/steady_profile.py "$T" "$O/steady_$M.txt" --skip 3 --title "$M N=1" && head -40 "$O/steady_$M.txt"
