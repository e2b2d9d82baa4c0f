set -o pipefail
O=gpurun_out/tkprof; mkdir -p $O
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tk -o tk -- python3 "$ROOT/bench/codec_bench.py" --sizes 25557032 --specs topk:0.01,threshold:0.02:0.05 --no-host) > $O/prof.log 2>&1 || exit 1
S=$(find /tmp/tk -name "tk_kernel_stats.csv" | head -1); cp "$S" $O/kernel_stats.csv
T=$(find /tmp/tk -name "tk_kernel_trace.csv" | head -1); cp "$T" $O/kernel_trace.csv
cut -d, -f1-8 $O/kernel_stats.csv | head -30
