# A/B: the end-of-backward join of the weight-gradient side stream deferred to the async PS's
# per-bucket encode waits (HIPPS_WGRAD_DEFER_JOIN=1), two interleaved rounds
set -o pipefail
O=gpurun_out/${1:-r5df}; mkdir -p $O
for r in 1 2; do
  for d in 0 1; do
    HIPPS_WGRAD_DEFER_JOIN=$d timeout -k 10 200 python bench.py --steps 30 --warmup 8 --out $O/defer${d}_r$r.json \
      > $O/defer${d}_r$r.log 2>&1 || exit 1
    echo "defer=$d round $r: $(python3 -c "import json;d=json.load(open('$O/defer${d}_r$r.json'));print(d['value'], d['ms_per_step'], d['final_loss'])")"
  done
done
