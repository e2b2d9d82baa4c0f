#!/bin/bash
# round-4: same-box A/Bs, two interleaved rounds each: the BN forward apply unroll
# (HIPPS_BN_APPLY_UNR=2 on the layer-1/2 tensors vs 1, with the fused-BN tests under it) and the
# forward-time drain of held gradients (HIPPS_HOLD_DRAIN, with the PS GPU tests)
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
HIPPS_BN_APPLY_UNR=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fused_bn.py tests/test_conv1x1_gpu.py > $O/tests_unr2.log 2>&1 || { tail -30 $O/tests_unr2.log; exit 1; }
tail -1 $O/tests_unr2.log
for r in 1 2; do
  for v in 2 1; do
    timeout -k 10 300 env HIPPS_BN_APPLY_UNR=$v python bench.py --steps 30 --warmup 5 --out $O/ab_unr${v}_r$r.json > $O/ab_unr${v}_r$r.log 2>&1 || { tail -20 $O/ab_unr${v}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_unr${v}_r$r.json'));print('unr$v r$r', d['value'], d['ms_per_step'], d['final_loss'])"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ps_async_gpu.py tests/test_fused_bn.py > $O/pstests.log 2>&1 || { tail -30 $O/pstests.log; exit 1; }
tail -1 $O/pstests.log
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 env HIPPS_HOLD_DRAIN=$v python bench.py --steps 30 --warmup 5 --out $O/ab_drain${v}_r$r.json > $O/ab_drain${v}_r$r.log 2>&1 || { tail -20 $O/ab_drain${v}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_drain${v}_r$r.json'));print('drain$v r$r', d['value'], d['ms_per_step'], d['final_loss'])"
  done
done
for v in 1 0; do
  HIPPS_HOST_TIMING=1 HIPPS_HOLD_DRAIN=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --out $O/alloc_drain$v.json > $O/alloc_drain$v.log 2>&1 || { tail -20 $O/alloc_drain$v.log; exit 1; }
  echo "drain=$v"; grep "host ms\|allocator" $O/alloc_drain$v.log
done
timeout -k 10 300 python -u tools/alloc_probe.py --out $O/alloc_probe.txt --steps 40 --warmup 5 > $O/alloc_probe.log 2>&1 || { tail -20 $O/alloc_probe.log; exit 1; }
head -40 $O/alloc_probe.txt
