#!/usr/bin/env python3
"""Per-layer kernel timings of the ResNet-50 headline step as the conv tuner measured them.

Runs two training steps of the bench configuration (batch 256, channels-last bf16, fused path,
mode='local') so every conv shape / epilogue goes through hipps.ops.nn.TUNER once, then prints each
tuned key with every candidate's time, the choice, and the roofline figures of the GEMM.

    python tools/tuner_dump.py --out gpurun_out/tuner.json
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import hipps
    from hipps.models import build_model
    from hipps.ops import nn as hnn

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    model = build_model("resnet50").to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    opt = hipps.SGD(model.named_parameters(), lr=0.1, momentum=0.9, mode="local", code="bf16", bf16_weights="on")
    for _ in range(2):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    rows = []
    tot_best = 0.0
    for key, t in hnn.TUNER.times.items():
        best = hnn.TUNER.cache[key]
        rows.append({"key": [str(k) for k in key], "choice": best, "ms": {k: round(v, 4) for k, v in t.items()}})
        tot_best += t[best]
    rows.sort(key=lambda r: -r["ms"][r["choice"]])
    for r in rows:
        print(r["choice"].ljust(12), f'{r["ms"][r["choice"]]:.4f}', " ".join(r["key"]),
              {k: v for k, v in r["ms"].items()})
    print(f"sum of chosen candidate times (one call per key): {tot_best:.3f} ms")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "sum_ms": tot_best}, f, indent=1)
    opt.close()


if __name__ == "__main__":
    main()
