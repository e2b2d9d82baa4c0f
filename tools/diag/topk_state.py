"""Diagnostic: run the top-k codec over a stream of fresh gradients (error feedback on) and print
the device selection state after each call: threshold key, speculative bound, pool use, full-pass
fallback flag, list length.  Layout mirrors SelState in hipps/csrc/topk.hip."""
import sys

import torch

sys.path.insert(0, ".")
from hipps import codecs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25557032
spec = sys.argv[2] if len(sys.argv) > 2 else "topk:0.01"
dev = torch.device("cuda")
c = codecs.get_codec(spec)
lay = c.layout(n)
buf = torch.empty(lay.nbytes, dtype=torch.uint8, device=dev)
views = lay.views(buf)
st = c.init_state(n, dev)
xs = [torch.randn(n, device=dev) * 1e-2 for _ in range(4)]
nchunks = (n + 4095) // 4096
cpw = (nchunks + 1023) // 1024
nreg = (nchunks + cpw - 1) // cpw
SEL = (8 + 24 + 256 + 8 * 2048) * 4  # prefix..prev_T, redo + pad, pool_used, hist copies
for step in range(12):
    c.encode_into(xs[step % 4], views, st)
    torch.cuda.synchronize()
    w = st["ws"][: SEL + 4 * (2 * nchunks + nreg)].cpu().view(torch.int32)
    hdr = w[:8].tolist()
    pool = [w[32 + 32 * s].item() for s in range(8)]
    ccnt = w[SEL // 4 + nchunks: SEL // 4 + 2 * nchunks]
    rcnt = w[SEL // 4 + 2 * nchunks: SEL // 4 + 2 * nchunks + nreg]
    print(f"step {step}: T={hdr[0]:#x} remaining={hdr[2]} capw={hdr[3]} pool_cap={hdr[4]} full={hdr[5]} "
          f"spec_lo={hdr[6]:#x} pool_used={pool} listed={int(rcnt.sum())} ({rcnt.sum().item() / n:.3%}) "
          f"max_region={int(rcnt.max())}", flush=True)
