# Same-box A/B of bench.py argument sets, two interleaved rounds:
#   bash tools/diag/arg_ab.sh <out> "<args A>" "<args B>" ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  i=0
  for a in "$@"; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 8 $a --out $O/v${i}_r$r.json > $O/v${i}_r$r.log 2>&1 || exit 1
    echo "[$a] round $r: $(python3 -c "import json;d=json.load(open('$O/v${i}_r$r.json'));print(d['value'], d['ms_per_step'])")"
    i=$((i+1))
  done
done
