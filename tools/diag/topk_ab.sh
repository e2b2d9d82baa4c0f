# Top-k / threshold encode variants: kernel tests under each, then the 25.6 M codec bench (cold
# MALL) twice per variant, interleaved
#   bash tools/diag/topk_ab.sh <out> "VAR=val ..." "VAR=val ..." ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for v in "$@"; do
  env $v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "topk or threshold" > $O/tests_$i.log 2>&1 || { echo "tests failed under [$v]"; tail -30 $O/tests_$i.log; exit 1; }
  echo "[$v] $(tail -1 $O/tests_$i.log)"; i=$((i+1))
done
for r in 1 2; do
  i=0
  for v in "$@"; do
    env $v timeout -k 10 200 python bench/codec_bench.py --sizes 1000000,25557032 \
      --specs topk:0.01,topk_bf16:0.01,threshold:0.02:0.05,threshold:0.1:0.05 --no-host > $O/bench_${i}_r$r.log 2>&1 || exit 1
    echo "[$v] r$r: $(python3 -c "
import json
for l in open('$O/bench_${i}_r$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['n'], d['codec'], d['encode_us'], end='; ')
")"; i=$((i+1))
  done
done
