# Generic same-box A/B of one environment switch on the headline bench, two interleaved rounds:
#   bash tools/diag/env_ab.sh <out> VAR valueA valueB [extra bench args...]
set -o pipefail
O=gpurun_out/$1; V=$2; A=$3; B=$4; shift 4
mkdir -p $O
for r in 1 2; do
  for val in "$A" "$B"; do
    env $V=$val timeout -k 10 200 python bench.py --steps 30 --warmup 8 "$@" --out $O/${V}_${val}_r$r.json \
      > $O/${V}_${val}_r$r.log 2>&1 || exit 1
    echo "$V=$val round $r: $(python3 -c "import json;d=json.load(open('$O/${V}_${val}_r$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
