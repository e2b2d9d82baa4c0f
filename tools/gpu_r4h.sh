#!/bin/bash
# round-4: validate the memory-path kernel changes (finalize load depth, max-pool loads, gemm2
# epilogue batches, top-k prefetch, int8 DPP rows) and measure them: kernel tests, the finalize
# probe at both depths, the tuner's per-layer table, a same-box bench A/B of the finalize depth
# (interleaved twice) and a steady kernel table of the default build
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gemm2_gpu.py tests/test_stem_gpu.py tests/test_conv1x1_gpu.py tests/test_fused_bn.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/bn_fin_probe.py --out $O/bn_fin_u12.json || exit 1
HIPPS_BN_FIN_U=4 timeout -k 10 120 python tools/bn_fin_probe.py --out $O/bn_fin_u4.json || exit 1
timeout -k 10 300 python tools/tuner_dump.py --out $O/tuner.json > $O/tuner.log 2>&1 || { tail -20 $O/tuner.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4h/tuner.json"))
for r in d["rows"][:14]:
    print(r["key"], r["choice"], {k: round(v, 3) for k, v in r["ms"].items()})
PY
for r in 1 2; do
  for v in 12 4; do
    timeout -k 10 300 env HIPPS_BN_FIN_U=$v python bench.py --steps 30 --warmup 5 --out $O/ab_fin${v}_r$r.json > $O/ab_fin${v}_r$r.log 2>&1 || { tail -20 $O/ab_fin${v}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_fin${v}_r$r.json'));print('fin$v r$r', d['value'], d['ms_per_step'], d['final_loss'])"
  done
done
STEPS=12 bash tools/gpu_prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
cp gpurun_out/prof/steady.txt $O/steady.txt
head -12 $O/steady.txt
grep -E "maxpool|finalize|k_gemm<.*, (6|10|26)," $O/steady.txt | cut -c1-150
