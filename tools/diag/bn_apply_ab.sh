# BN forward apply bandwidth, UNR 1 vs 2 (tools/bench_bn_apply.py)
set -o pipefail
O=gpurun_out/${1:-r5bn}; mkdir -p $O
for u in 1 2; do
  HIPPS_BN_APPLY_UNR=$u timeout -k 10 200 python tools/bench_bn_apply.py --out $O/bn_apply_unr$u.json > $O/bn_apply_unr$u.log 2>&1 || exit 1
  echo "== UNR $u"; cat $O/bn_apply_unr$u.log | grep -v amdgpu.ids
done
