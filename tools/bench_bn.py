"""Microbenchmark: fused BN(+res)(+relu) fwd/bwd vs eager (MIOpen BN + elementwise) per ResNet-50 shape."""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops.nn import FusedBatchNorm2d  # noqa: E402

SHAPES = [(256, 64, 112, 112), (256, 64, 56, 56), (256, 256, 56, 56), (256, 128, 28, 28), (256, 512, 28, 28),
          (256, 256, 14, 14), (256, 1024, 14, 14), (256, 512, 7, 7), (256, 2048, 7, 7)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


out = []
for shape in SHAPES:
    N, C, H, W = shape
    for res in (False, True):
        x = torch.randn(shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        g = torch.randn_like(x)
        row = {"shape": shape, "res": res}
        for fused in (True, False):
            m = FusedBatchNorm2d(C, relu=True, fused=fused).cuda()
            xx = x.clone().requires_grad_(True)

            def fwd():
                return m(xx, residual=r)

            def fb():
                y = m(xx, residual=r)
                y.backward(g)

            tf = timeit(fwd)
            tfb = timeit(fb)
            gb = x.numel() * 2 / 1e9
            row["fused" if fused else "eager"] = {"fwd_ms": round(tf, 3), "fwdbwd_ms": round(tfb, 3),
                                                   "GB_per_pass": round(gb, 3)}
        print(json.dumps(row), flush=True)
        out.append(row)
json.dump(out, open(os.path.join(ROOT, "gpurun_out/bench_bn.json"), "w"), indent=1)
