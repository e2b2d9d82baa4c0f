# Llama-3-8B (config 5) at N=1: native vs Python PS loop (host timing), or with "prof" a
# steady-state kernel profile of each
#   bash tools/diag/llama8b_ab.sh <out> [prof]
set -o pipefail
O=gpurun_out/${1:-r5y}; mkdir -p $O
A="--model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4"
if [ "${2:-}" = "prio" ]; then  # the PS stream at the worker's priority (HIPPS_PS_PRIORITY=0)
  for L in 1 0; do
    HIPPS_HOST_TIMING=1 HIPPS_PS_PRIORITY=0 HIPPS_NATIVE_PS=$L timeout -k 10 400 python bench.py $A --steps 6 --warmup 3 \
      --out $O/l8_prio0_native$L.json > $O/l8_prio0_native$L.log 2>&1 || exit 1
    echo "native=$L prio0: $(grep -h 'host ms' $O/l8_prio0_native$L.log)"; cut -c1-150 $O/l8_prio0_native$L.json
  done
  exit 0
fi
if [ "${2:-}" != "prof" ]; then
  HIPPS_HOST_TIMING=1 timeout -k 10 400 python bench.py $A --steps 6 --warmup 3 --out $O/l8_native.json \
    > $O/l8_native.log 2>&1 &&
  grep -h "host ms" $O/l8_native.log && cut -c1-150 $O/l8_native.json &&
  HIPPS_HOST_TIMING=1 HIPPS_NATIVE_PS=0 timeout -k 10 400 python bench.py $A --steps 6 --warmup 3 \
    --out $O/l8_python.json > $O/l8_python.log 2>&1 &&
  grep -h "host ms" $O/l8_python.log && cut -c1-150 $O/l8_python.json
  exit $?
fi
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for L in 1 0; do
  (cd /tmp && HIPPS_NATIVE_PS=$L timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/l8prof$L -o l8 -- python3 "$ROOT/bench.py" $A --steps 6 --warmup 3) > $O/l8_prof$L.log 2>&1 || exit 1
  T=$(find /tmp/l8prof$L -name "l8_kernel_trace.csv" | head -1)
  python3 tools/steady_profile.py "$T" "$O/steady_l8_native$L.txt" --skip 3 --title "Llama-3-8B N=1 native_ps=$L" &&
  head -16 "$O/steady_l8_native$L.txt" || exit 1
done
