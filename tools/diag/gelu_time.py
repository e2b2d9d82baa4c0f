"""Time the BERT-base MLP GEMMs with the GELU epilogues (gemm2 kGelu / kGeluB) against hipBLASLt +
PyTorch's GELU kernels, every gemm2 tile, same process (the tuner's own candidate sets).

    python tools/diag/gelu_time.py [--M 16384] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hipps.ops.nn as hnn  # noqa: E402
from hipps.ops._native import native  # noqa: E402


def _time(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return round(sorted(ts)[n // 2], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--F", type=int, default=3072)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    C = native()
    M, D, F4 = a.M, a.D, a.F
    dev = "cuda"
    x = torch.randn(M, D, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(F4, D, device=dev) * 0.03).to(torch.bfloat16)
    b1 = torch.randn(F4, device=dev) * 0.1
    w2 = (torch.randn(D, F4, device=dev) * 0.03).to(torch.bfloat16)
    w2t = w2.t().contiguous()
    dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
    pre = torch.empty(M, F4, device=dev, dtype=torch.bfloat16)
    post = torch.empty_like(pre)
    out = {}

    def fwd_blas():
        torch.addmm(b1.to(torch.bfloat16), x, w1.t(), out=pre)
        torch._C._nn.gelu(pre, out=post)

    def fwd_mm_only():
        torch.addmm(b1.to(torch.bfloat16), x, w1.t(), out=pre)

    row = {"blas(addmm+gelu)": _time(fwd_blas), "addmm only": _time(fwd_mm_only)}
    for name in hnn._g2_names(F4) + ["g2_256x256s6", "g2_256x128", "g2_256x128s3"]:
        bm, bn, ns = hnn._g2_parse(name)
        row[name] = _time(lambda: C.gemm2_conv(x, w1, post, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns,
                                               bias=b1, gelu_pre=pre, gelu=1))
        row[name + " nogelu"] = _time(lambda: C.gemm2_conv(x, w1, post, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn,
                                                           stages=ns, bias=b1))
    out["gelu_fwd"] = row
    print("gelu_fwd", row, flush=True)

    dpre = torch.empty(M, F4, device=dev, dtype=torch.bfloat16)

    def bwd_blas():
        return torch.ops.aten.gelu_backward(torch.mm(dy, w2), pre)

    row = {"blas(mm+gelu_bwd)": _time(bwd_blas), "mm only": _time(lambda: torch.mm(dy, w2)),
           "transpose": _time(lambda: w2.t().contiguous())}
    for name in hnn._g2_names(F4) + ["g2_256x256s6", "g2_256x128", "g2_256x128s3"]:
        bm, bn, ns = hnn._g2_parse(name)
        row[name] = _time(lambda: C.gemm2_conv(dy, w2t, dpre, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns,
                                               gelu_pre=pre, gelu=2))
    out["gelu_dgrad"] = row
    print("gelu_dgrad", row, flush=True)

    # the MLP input gradient with the residual gradient: dx = dpre w1 + dy
    w1t = w1.t().contiguous()
    dx = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    row = {"addmm(dy, dpre, w1)": _time(lambda: torch.addmm(dy, dpre, w1)),
           "mm + add": _time(lambda: torch.mm(dpre, w1).add_(dy)), "mm only": _time(lambda: torch.mm(dpre, w1))}
    for name in hnn._g2_names(D) + ["g2_256x256s6", "g2_256x128", "g2_256x128s3"]:
        bm, bn, ns = hnn._g2_parse(name)
        row[name + " kAdd"] = _time(lambda: C.gemm2_conv(dpre, w1t, dx, None, dy, None, 1, 1, 1, 1, 1, 0, bm, bn,
                                                         stages=ns))
    out["mlp_dx"] = row
    print("mlp_dx", row, flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
