#!/usr/bin/env python3
"""Run one gemm2 kernel configuration repeatedly (for rocprofv3 --pmc passes).

    python tools/g2_one.py conv 256,14,256,1 --tile 256x256 --iters 20    # 3x3: Cin,H,Cout,stride
    python tools/g2_one.py wgrad 128,28,128,1,3 --cfg 0 --iters 20         # Cin,H,Cout,stride,k
    python tools/g2_one.py gemm 50176,1024,512 --tile 128x128 --iters 20  # M,K,N
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops._native import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["conv", "wgrad", "gemm"])
    ap.add_argument("shape")
    ap.add_argument("--tile", default="128x128")
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = native()
    cl = torch.channels_last
    bm, bn = (int(v) for v in a.tile.split("x"))
    v = [int(t) for t in a.shape.split(",")]
    torch.manual_seed(0)
    if a.kind == "gemm":
        M, K, N = v
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fn = lambda: C.gemm2_conv(x, w, y, None, None, None, M, 1, bm=bm, bn=bn, stages=a.stages)  # noqa: E731
    elif a.kind == "conv":
        cin, h, cout, st = v
        x = torch.randn(256, cin, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=cl)
        ho = (h + 2 - 3) // st + 1
        y = torch.empty(256, cout, ho, ho, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        fn = lambda: C.gemm2_conv(x, w, y, None, None, None, h, h, st, 3, 3, 1, bm, bn, stages=a.stages)  # noqa: E731
    else:
        cin, h, cout, st, k = v
        pad = k // 2
        ho = (h + 2 * pad - k) // st + 1
        x = torch.randn(256, cin, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(256, cout, ho, ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        dw = torch.empty(cout, cin, k, k, device="cuda").contiguous(memory_format=cl)
        fn = lambda: C.gemm2_wgrad(dy, x, dw, k, k, st, pad, h, h, a.cfg, a.stages)  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{a.kind} {a.shape} {a.tile} cfg{a.cfg} s{a.stages}: {s.elapsed_time(e) / a.iters:.4f} ms")


if __name__ == "__main__":
    main()
