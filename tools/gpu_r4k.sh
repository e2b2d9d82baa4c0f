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
# allocator growth (profiles/r4/r4j: ~2.4 new activation-sized segments per step on the main stream):
# without the weight-gradient side stream (its record_stream'd inputs), and with expandable segments
for v in nows expand; do
  case $v in
    nows) E="HIPPS_WGRAD_STREAM=0";;
    expand) E="PYTORCH_HIP_ALLOC_CONF=expandable_segments:True";;
  esac
  timeout -k 10 300 env $E python -u tools/alloc_probe.py --out $O/alloc_probe_$v.txt --steps 40 --warmup 5 > $O/alloc_probe_$v.log 2>&1 || { tail -20 $O/alloc_probe_$v.log; exit 1; }
  echo "== $v"; head -12 $O/alloc_probe_$v.txt
done
