#!/bin/bash
# round-4: direct-from-slot PS update (M = 1) and BN-prologue side-stream weight gradient --
# their GPU tests, then a same-box A/B (interleaved twice)
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ps_async_gpu.py tests/test_fused_bn.py tests/test_stem_gpu.py tests/test_conv1x1_gpu.py tests/test_resnet_trajectory_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 env HIPPS_PS_DIRECT=$v python bench.py --steps 30 --warmup 5 --out $O/ab_direct${v}_r$r.json > $O/ab_direct${v}_r$r.log 2>&1 || { tail -20 $O/ab_direct${v}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_direct${v}_r$r.json'));print('direct$v r$r', d['value'], d['ms_per_step'], d['final_loss'], d['ps'].get('direct_updates'))"
  done
done
STALL_OUT=$O/stall bash tools/gpu_stall.sh > /dev/null || exit 1
grep -A1 "host lead" $O/stall/stalls.txt
timeout -k 10 120 python tools/bn_fin_probe.py --out $O/bn_fin_u12.json || exit 1
HIPPS_BN_FIN_U=4 timeout -k 10 120 python tools/bn_fin_probe.py --out $O/bn_fin_u4.json || exit 1
timeout -k 10 300 python tools/tuner_dump.py --out $O/tuner.json > $O/tuner.log 2>&1 || { tail -20 $O/tuner.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4g/tuner.json"))
for r in d["rows"][:12]:
    print(r["key"], r["choice"], {k: round(v, 3) for k, v in r["ms"].items()})
PY
