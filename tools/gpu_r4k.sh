#!/bin/bash
# round-4: stream-priority A/B (two interleaved rounds): default (PS stream high, training on the
# default stream); the training step on a high-priority stream (BENCH_HIPRIO=1: the weight-gradient
# and comm streams then rank below it); the PS stream at the default priority (HIPPS_PS_PRIORITY=0)
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
for r in 1 2; do
  for v in base hiprio psprio0; do
    case $v in
      base) E="";;
      hiprio) E="BENCH_HIPRIO=1";;
      psprio0) E="HIPPS_PS_PRIORITY=0";;
    esac
    timeout -k 10 300 env $E python bench.py --steps 30 --warmup 5 --out $O/ab_${v}_r$r.json > $O/ab_${v}_r$r.log 2>&1 || { tail -20 $O/ab_${v}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_${v}_r$r.json'));print('$v r$r', d['value'], d['ms_per_step'], d['final_loss'], d['ps'].get('drops'), d.get('ps_staleness_mean'))"
  done
done
