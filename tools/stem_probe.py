"""Run the hipps stem kernels (forward with statistics, weight gradient) on the ResNet-50 shape a
few times -- a target for rocprofv3 --kernel-trace / --pmc.  python tools/stem_probe.py [--iters N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipps.ops._native import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    cl = torch.channels_last
    n = a.batch
    x = torch.randn(n, 3, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn(64, 3, 7, 7, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    y = torch.empty(n, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    part = torch.empty(2, 64, native().stem_mtiles(n, 112), device="cuda")
    dy = torch.randn_like(y)
    dw = torch.empty(64, 3, 7, 7, device="cuda").contiguous(memory_format=cl)
    for _ in range(a.iters):
        native().stem_forward(x, w, y, part)
        native().stem_wgrad(dy, x, dw)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
