#!/bin/bash
# N=8 readiness on ONE GPU (VERDICT r2 task 2):
#  1. N=1 bench (same-box baseline)
#  2. --emulate-remote 7: one process; the co-located PS also accumulates 7 emulated remote
#     messages per step and sweeps their push / pull bytes (upper bound of the PS cost at N=8)
#  3. the same with HIPPS_TRACE=1 (PS accumulate / update device time per step)
#  4. --emulate-workers 7: 8 ranks on cuda:0 (gloo rendezvous), the real W=8 control block;
#     ranks 1..7 push zero gradients + pull in lockstep with worker 0 (protocol rehearsal; its
#     timing includes 8 HIP contexts time-sharing one GPU)
#  5. dedicated-PS topology (rank 0 only serves) with 3 ranks sharing the GPU
#  LAT=1: only the PS update latency runs (HIPPS_PS_LATENCY=1: GPU time from worker 0's push
#     doorbell of a bucket to the publish that includes it), whole-model vs per-bucket versions,
#     at N=1 and under --emulate-remote 7
set -o pipefail
O=gpurun_out/emu
mkdir -p $O
T="timeout -k 10 400"
if [ "${LAT:-0}" = 1 ]; then
  for g in model bucket; do
    for e in 0 7; do
      HIPPS_PS_LATENCY=1 HIPPS_PS_GRANULARITY=$g $T python -u bench.py --steps 30 --warmup 8 --emulate-remote $e \
        --out $O/lat_${g}_er$e.json > $O/lat_${g}_er$e.log 2>&1 || { tail -30 $O/lat_${g}_er$e.log; exit 1; }
      python -c "
import json; r = json.load(open('$O/lat_${g}_er$e.json')); p = r['ps']
print('$g', 'er$e', r['value'], r['ms_per_step'], 'stale', r.get('ps_staleness_mean'), r.get('loss_every5'),
      {k: v for k, v in p.items() if k.startswith('push_to')})"
    done
  done
  exit 0
fi
$T python -u bench.py --steps 30 --warmup 8 --out $O/n1.json > $O/n1.log 2>&1 || { tail -30 $O/n1.log; exit 1; }
$T python -u bench.py --steps 30 --warmup 8 --emulate-remote 7 --out $O/er7.json > $O/er7.log 2>&1 || { tail -30 $O/er7.log; exit 1; }
HIPPS_TRACE=1 $T python -u bench.py --steps 30 --warmup 8 --emulate-remote 7 --out $O/er7_trace.json > $O/er7_trace.log 2>&1 || { tail -30 $O/er7_trace.log; exit 1; }
HIPPS_TRACE=1 $T python -u bench.py --steps 30 --warmup 8 --out $O/n1_trace.json > $O/n1_trace.log 2>&1 || { tail -30 $O/n1_trace.log; exit 1; }
export HIPPS_BACKEND=gloo
$T python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29711 \
   bench.py --gpus 8 --steps 30 --warmup 8 --emulate-workers 7 --out $O/emu7.json > $O/emu7.log 2>&1 || { tail -40 $O/emu7.log; exit 1; }
$T python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29713 \
   bench.py --gpus 3 --steps 10 --warmup 3 --batch 64 --ps-dedicated --out $O/ded3.json > $O/ded3.log 2>&1 || { tail -40 $O/ded3.log; exit 1; }
python - <<'PY'
import json
for k in ("n1", "er7", "er7_trace", "n1_trace", "emu7", "ded3"):
    r = json.load(open(f"gpurun_out/emu/{k}.json"))
    print(k, r["value"], r["ms_per_step"], "stale", r.get("ps_staleness_mean"), "loss", r.get("loss_every5"),
          "trace", r.get("trace_device_ms_per_step"), "acc_launches", r["ps"].get("acc_launches"))
PY
