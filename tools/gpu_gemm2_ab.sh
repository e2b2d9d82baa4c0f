#!/bin/bash
# gemm2 numerics tests + N=1 bench A/B (HIPPS_GEMM2=1 vs 0) + steady kernel profile
set -o pipefail
O=gpurun_out/g2
mkdir -p $O gpurun_out/prof
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/bench_g2.json > $O/bench_g2.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_g2.log; exit 1; }
HIPPS_GEMM2=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/bench_g1.json > $O/bench_g1.log 2>&1 || { echo "bench g1 failed"; tail -30 $O/bench_g1.log; exit 1; }
python - <<'PY'
import json
for k in ("bench_g2", "bench_g1"):
    r = json.load(open(f"gpurun_out/g2/{k}.json"))
    print(k, r["value"], r["ms_per_step"], r["loss_every5"])
PY
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/hprof -o bench -- python3 $ROOT/bench.py --steps 12 --warmup 5 > $ROOT/gpurun_out/prof/bench_prof.log 2>&1 || { echo "prof failed"; exit 1; }
cd $ROOT
T=$(find /tmp/hprof -name "bench_kernel_trace.csv" | head -1)
python3 tools/steady_profile.py "$T" gpurun_out/prof/steady.txt --skip 5 --title "ResNet-50 bs256 ps_async bf16 N=1 (gemm2)"
head -40 gpurun_out/prof/steady.txt
