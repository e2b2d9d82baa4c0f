#!/bin/bash
# round-4: what async costs and buys at N=1 -- headline-config loss trajectories of local, plain
# AsySG-InCon (model / bucket granularity) and the look-ahead variants; same-box bench A/B of the
# publication granularity and bucket size (interleaved twice)
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u tools/trajectory.py --headline --runs local,async,async_la,async_bucket,async_bucket_la \
  --out $O/traj_headline.json > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
grep -o '"variant": "[a-z_]*"' $O/traj.log
for r in 1 2; do
  for cfg in "model 64" "bucket 16" "bucket 64" "bucket 8"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --granularity $1 --bucket-mb $2 --out $O/ab_${1}_${2}_r$r.json > $O/ab_${1}_${2}_r$r.log 2>&1 || { tail -20 $O/ab_${1}_${2}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_${1}_${2}_r$r.json'));print('$1 $2 r$r', d['value'], d['ms_per_step'], d['final_loss'], d['ps_staleness_mean'])"
  done
done
