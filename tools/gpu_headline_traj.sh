#!/bin/bash
# Headline-config convergence bisect (VERDICT r2 task 1): ResNet-50, batch 256, bf16 wire, auto
# bf16 weight shadow, lr 0.1, momentum 0.9, wd 5e-5, 60 steps on one fixed synthetic batch.
# KTESTS=1 first runs the fused-optimizer kernel tests; BENCH=1 adds a 30-step N=1 bench.
set -o pipefail
O=gpurun_out/htraj
mkdir -p $O
T="timeout -k 10 300"
RUNS=${RUNS:-local,async_md0,async,local+code=fp32+bf16_weights=off,async+code=fp32+bf16_weights=off}
if [ -n "$KTESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
      -k "sgd or adam or chunk or lookahead or masked" > $O/ktests.log 2>&1 || { tail -30 $O/ktests.log; exit 1; }
  tail -2 $O/ktests.log
fi
$T python -u tools/trajectory.py --headline --runs $RUNS --out $O/hipps.json > $O/hipps.log 2>&1 || { tail -30 $O/hipps.log; exit 1; }
if [ -z "$NOPLAIN" ]; then
  $T python -u tools/trajectory.py --headline --plain --out $O/plain.json > $O/plain.log 2>&1 || { tail -30 $O/plain.log; exit 1; }
fi
if [ -n "$BENCH" ]; then
  $T python -u bench.py --steps 30 --warmup 8 --out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
  cut -c1-400 $O/bench.json
fi
python - <<'PY'
import json
for f in ["gpurun_out/htraj/hipps.json", "gpurun_out/htraj/plain.json"]:
    try:
        recs = json.load(open(f))
    except Exception:
        continue
    for r in recs:
        L = r["losses"]
        print(r["variant"][:40].ljust(40), " ".join(f"{x:.2f}" for x in L[::4]), "| min-after-20 ratio",
              round(max(L[i] / min(L[:i + 1]) for i in range(20, len(L))), 3))
PY
