# A/B of the top-k / threshold collect prefetch (HIPPS_TOPK_PF) at 25.6 M, cold MALL, plus the
# threshold message's count after the timed calls (saturation check)
set -o pipefail
O=gpurun_out/${1:-tkpf}; mkdir -p $O
for pf in ${PFS:-1 0 1 0}; do
  HIPPS_TOPK_PF=$pf timeout -k 10 200 python bench/codec_bench.py --sizes 25557032 --specs ${SPECS:-topk:0.01,threshold:0.02:0.05} \
    --no-host > $O/pf$pf.log 2>&1 || exit 1
  echo "PF=$pf: $(python3 -c "
import json
for l in open('$O/pf$pf.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['codec'], d['encode_us'], end='; ')
")"
done
timeout -k 10 120 python - <<'PY'
import torch, sys
sys.path.insert(0, ".")
from hipps import codecs
n = 25557032
for spec in "${TSPECS:-threshold:0.02:0.05}".split(","):
  c = codecs.get_codec(spec)
  lay = c.layout(n); buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda"); v = lay.views(buf)
  st = c.init_state(n, "cuda")
  xs = [torch.randn(n, device="cuda") * 1e-2 for _ in range(4)]
  for i in range(40):
    c.encode_into(xs[i % 4], v, st)
    if i in (0, 1, 4, 10, 39):
        torch.cuda.synchronize()
        r = st["resid"]
        print(f"{spec} call {i}: count {int(v['count'][0])} cap {c.cap_of(n)} |resid|>tau {(r.abs() > c.tau).float().mean().item():.3f}", flush=True)
PY
