#!/bin/bash
# Round-3 GPU check: gemm2 probe, the new GPU tests (per-chunk steps, look-ahead, bucket pulls)
set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u tools/gemm2_probe.py --out gpurun_out/g2/probe.json > gpurun_out/g2/probe.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/g2/probe.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open("gpurun_out/g2/probe.json")):
    keys = [k for k in r if k.endswith("_TF")]
    print({k: r[k] for k in ("M", "K", "N", "Cin", "H", "Cout", "stride") if k in r}, {k: r[k] for k in keys})
PY
timeout -k 10 400 python -u -m pytest tests/test_ps_async_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "bucket or chunk or lookahead" > gpurun_out/g2/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/g2/tests.log; exit 1; }
tail -2 gpurun_out/g2/tests.log
