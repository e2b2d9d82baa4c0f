"""Achieved HBM bandwidth of the fused BN forward apply (norm.hip k_bn_apply_fwd) on the ResNet-50
bs256 shapes: y = relu(x * scale + shift [+ res]) over channels-last bf16, bytes = read x (+ res)
+ write y.  Run once per HIPPS_BN_APPLY_UNR setting (read at the first call).

    python tools/bench_bn_apply.py [--out file.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipps.ops._native import native  # noqa: E402

SHAPES = [(256, 64, 112, 112), (256, 64, 56, 56), (256, 256, 56, 56), (256, 128, 28, 28), (256, 512, 28, 28),
          (256, 256, 14, 14), (256, 1024, 14, 14), (256, 512, 7, 7), (256, 2048, 7, 7)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C_ = native()
    rows = []
    cl = torch.channels_last
    for shape in SHAPES:
        n, c, h, w = shape
        x = torch.randn(shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        sc, sh = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.1
        for res in (False, True):
            r = torch.randn_like(x) if res else None
            y = torch.empty_like(x)
            fn = lambda: C_.bn_apply(x, r, y, sc, sh, c, True)  # noqa: E731
            for _ in range(3):
                fn()
            flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
            ts = []
            for _ in range(a.iters):
                flush.zero_()  # (the 256 MB MALL: every call starts cold)
                s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                s.record()
                fn()
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            us = sorted(ts)[len(ts) // 2]
            nbytes = x.numel() * 2 * (3 if res else 2)
            rows.append({"shape": shape, "res": res, "us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)})
            print(rows[-1], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"unr": os.environ.get("HIPPS_BN_APPLY_UNR", "1"), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
