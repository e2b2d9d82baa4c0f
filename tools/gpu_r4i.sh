#!/bin/bash
# round-4: same-box A/B of the BN forward apply unroll (HIPPS_BN_APPLY_UNR=2 on the layer-1/2
# tensors vs 1), two interleaved rounds, with the fused-BN tests under the unrolled kernel
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
