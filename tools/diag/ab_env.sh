# Same-box A/B of one environment switch on the headline bench, interleaved.
#   bash tools/diag/ab_env.sh <out-dir> <VAR> <value-A> <value-B> [rounds] [bench args...]
set -o pipefail
O=gpurun_out/$1; V=$2; A=$3; B=$4; R=${5:-2}; shift 5 2>/dev/null || shift $#
mkdir -p $O
for r in $(seq 1 $R); do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py "$@" --out $O/b_${val}_$r.json > $O/b_${val}_$r.log 2>&1 || { echo "fail $V=$val"; tail -20 $O/b_${val}_$r.log; exit 1; }
    echo "$V=$val run $r $(grep -o '"value": [0-9.]*' $O/b_${val}_$r.json)"
  done
done
