"""Rank-0 HBM budget of the async PS for a model / world size, without allocating anything.

    python tools/ps_budget.py --model llama3-8b --workers 8 [--dedicated] [--optim adam]

Prints every term of hipps.parallel.ps_async.ps_memory_budget (mailbox, publish buffers, master,
accumulator, optimizer state; co-located worker 0's parameters, gradients, bf16 shadow, wire and
codec state) against one MI355X's 288 GB, as JSON.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipps.parallel.ps_async import budget_for_shapes  # noqa: E402

HBM = 288 * 10**9


def shapes_of(name):
    from hipps.models import resnet50, transformer

    with torch.device("meta"):
        m = resnet50() if name == "resnet50" else transformer.build(name)
    return [tuple(p.shape) for p in m.parameters()]


def main():
    from hipps.config import PSConfig

    d = PSConfig()
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--codec", default="bf16")
    ap.add_argument("--bucket-mb", type=float, default=d.bucket_mb)
    ap.add_argument("--mailbox-mb", type=float, default=d.mailbox_mb)
    ap.add_argument("--mailbox-slots", type=int, default=d.mailbox_slots)
    ap.add_argument("--npub", type=int, default=d.npub, help="0 = auto (the engine's plan_geometry)")
    ap.add_argument("--hbm-gb", type=float, default=HBM / 1e9, help="rank 0's HBM; 0 = no limit (full geometry)")
    ap.add_argument("--param-wire", default="bf16")
    ap.add_argument("--optim", default="sgd", choices=["sgd", "adam"])
    ap.add_argument("--dedicated", action="store_true")
    a = ap.parse_args()
    b = budget_for_shapes(shapes_of(a.model), a.workers, a.codec, a.bucket_mb, a.mailbox_mb, a.mailbox_slots,
                          a.param_wire, 1 if a.optim == "sgd" else 2, a.dedicated, npub=a.npub,
                          hbm_bytes=int(a.hbm_gb * 1e9) if a.hbm_gb > 0 else None)
    keep = ("buckets", "mailbox_slots", "npub", "fits")
    gb = {k: (round(v / 1e9, 2) if k not in keep else v) for k, v in b.items()}
    gb["fits_288GB_before_activations"] = b["total"] < HBM
    gb["fits_270GB"] = b["total"] <= 270e9
    print(json.dumps({"model": a.model, "workers": a.workers, "codec": a.codec, "optim": a.optim,
                      "dedicated": a.dedicated, "param_wire": a.param_wire, "bucket_mb": a.bucket_mb,
                      "npub_arg": a.npub, "GB": gb}, indent=1))


if __name__ == "__main__":
    main()
