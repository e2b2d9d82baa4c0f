#!/usr/bin/env python3
"""Time the dual-BN backward (norm.hip bn_dual_backward) on the ResNet-50 downsample shapes for
each row-unroll depth, with the bytes it moves; and the single-BN backward apply for comparison.

    python tools/bench_bn_dual.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops._native import native  # noqa: E402


def main():
    C = native()
    cl = torch.channels_last
    for c, h in ((256, 56), (512, 28), (1024, 14), (2048, 7)):
        n = 256
        M = n * h * h
        mk = lambda: torch.randn(n, c, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)  # noqa: E731
        dz, x3, xd = mk(), mk(), mk()
        mask = torch.randint(0, 256, (M * c // 8,), dtype=torch.uint8, device="cuda")
        v = [torch.rand(c, device="cuda") + 0.5 for _ in range(6)]
        dx3, dxd = torch.empty_like(x3), torch.empty_like(xd)
        g = [torch.empty(c, device="cuda") for _ in range(4)]
        nbytes = M * c * (2 * 3 + 2 + 2 + 2 + 2 + 0.25)  # pass 1: dz x3 xd -> dx3; pass 2: dz xd -> dxd (+ bits x2)
        for unr in (2, 4, 8):
            fn = lambda: C.bn_dual_backward(None, 0, dz, x3, xd, mask, v[0], v[1], v[2], v[3], v[4], v[5], dx3, dxd,  # noqa: E731
                                            g[0], g[1], g[2], g[3], c, unr)
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 10
            print(f"C={c} H={h} unr={unr}: {ms * 1e3:.1f} us (incl. bn3 reduce), {nbytes / ms / 1e9:.2f} TB/s-equivalent",
                  flush=True)


def apply_bwd():
    """bn_backward_partials (finalize + apply, MASK_X) on the bn1 / bn2 shapes, 2 vs 4 vectors in
    flight per lane."""
    C = native()
    cl = torch.channels_last
    for c, h in ((64, 56), (128, 56), (128, 28), (256, 14), (512, 7)):
        n = 256
        M = n * h * h
        mk = lambda: torch.randn(n, c, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)  # noqa: E731
        dy, x = mk(), mk()
        v = [torch.rand(c, device="cuda") + 0.5 for _ in range(5)]
        part = torch.randn(2, c, 64, device="cuda")
        dx = torch.empty_like(x)
        g = [torch.empty(c, device="cuda") for _ in range(2)]
        for unr in (2, 4):
            fn = lambda: C.bn_backward_partials(part, 64, dy, x, 1, v[0], v[1], v[2], v[3], v[4], dx, None, g[0], g[1],  # noqa: E731
                                                c, None, unr)
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(20):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 20
            print(f"apply_bwd C={c} H={h} unr={unr}: {ms * 1e3:.1f} us, {M * c * 6 / ms / 1e9:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
    apply_bwd()
