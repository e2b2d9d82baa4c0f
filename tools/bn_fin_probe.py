"""Time the BatchNorm finalize kernels (partials -> per-channel coefficients) at ResNet-50's
partial-array shapes, with the partials evicted from L2 between calls as in the step (the producer
GEMM wrote them, then other work ran).

    python tools/bn_fin_probe.py [--out F]          # HIPPS_BN_FIN_U=4: the round-3 load depth

Shapes: (C, nrb) with nrb = M / 128 for the 1x1-GEMM epilogue partials (layer1: M = 802,816) and the
k_bn_reduce partial counts.  Prints one JSON object: us per call (median of 50) per shape.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipps.ops._native import native  # noqa: E402

SHAPES = [(64, 6272), (256, 6272), (128, 1568), (512, 1568), (256, 392), (1024, 392), (512, 98), (2048, 98)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    C_ = native()
    dev = torch.device("cuda:0")
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)  # > 8 x 4 MB L2
    res = {"fin_u": os.environ.get("HIPPS_BN_FIN_U", "12"), "shapes": {}}
    for c, nrb in SHAPES:
        part = torch.randn(2, c, nrb, device=dev)
        w = torch.rand(c, device=dev) + 0.5
        mean = torch.randn(c, device=dev)
        inv = torch.rand(c, device=dev) + 0.5
        dw = torch.empty(c, device=dev)
        db = torch.empty(c, device=dev)
        coef = torch.empty(3, c, device=dev)
        ts = []
        for it in range(a.iters + 5):
            flush.add_(1)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            C_.bn_finalize_bwd_partials(part, nrb, nrb * 128, w, mean, inv, dw, db, coef)
            e.record()
            e.synchronize()
            if it >= 5:
                ts.append(s.elapsed_time(e) * 1e3)
        # numerics against fp64 torch
        pa, pb = part[0].double().sum(1), part[1].double().sum(1)
        err = max((db.double() - pa).abs().max().item(), (dw.double() - pb).abs().max().item())
        res["shapes"][f"{c}x{nrb}"] = {"us": round(statistics.median(ts), 2), "max_abs_err": err}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
