#!/usr/bin/env python3
"""Loss trajectory of ResNet training on ONE fixed synthetic batch (convergence check).

Run it once with the hipps fusions on and once with ``--plain`` (every HIPPS_FUSED_* / conv
switch off and ``torch.optim.SGD`` instead of the fused hipps optimizer): the two per-step loss
curves must agree, and both must fall.  The switches are read at import time, so the plain
variant runs in its own process (tests/test_resnet_trajectory_gpu.py spawns both).

``--runs`` trains several hipps configurations in one process from the same init and batch:
  local          mode='local'
  async_md<k>    mode='ps_async', max_delay=k (N=1: rank 0 is PS and worker)
  async          mode='ps_async', max_delay=-1 (free-running AsySG-InCon, the reference's algorithm,
                 with the library defaults: per-bucket versions, 16 MB buckets)
  async_model    as async, whole-model versions (ps_granularity='model')
  async_la       as async, with the look-ahead publish (stale_lookahead=-1, delay compensation)
  async_model_la async_model with the look-ahead publish
  async_bucket   as async with per-bucket versions and 16 MB buckets spelled out
  async_slr      as async, with staleness-aware gradient scaling
  async_prefetch as async, with the host-chosen prefetch/direct pull instead of the GPU pull
  async_mc       as async, with delay-compensated momentum (``stale_momentum='comp'``)
A run name may carry ``+key=value`` overrides of the hipps.SGD keywords, e.g.
``local+code=fp32+bf16_weights=off`` (bisects the bf16 wire and the bf16 weight shadow).

``--headline`` is the exact bench.py configuration (BASELINE.json headline): batch 256, bf16 wire,
auto bf16 weight shadow, wd 5e-5, average=True, lr 0.1, momentum 0.9, 60 steps.

    python tools/trajectory.py --runs local,async_md0,async --out a.json
    python tools/trajectory.py --plain --out b.json
    python tools/trajectory.py --headline --runs local,async_md0,async --out h.json
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

PLAIN_ENV = {"HIPPS_FUSED_BN": "0", "HIPPS_FUSED_CONV": "0", "HIPPS_FUSED_GRAD": "0", "HIPPS_FUSED_POOL": "0",
             "HIPPS_FUSED_BNGRAD": "0", "HIPPS_FUSED_WGRAD": "0", "HIPPS_CONV_WGRAD": "0", "HIPPS_DGRAD_FWD": "0",
             "HIPPS_OWN_KXK": "0", "HIPPS_FUSED_PRO": "0"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--wd", type=float, default=5e-5)
    ap.add_argument("--runs", default="local")
    ap.add_argument("--codec", default="fp32")
    ap.add_argument("--bf16-weights", default="off", choices=["on", "off", "auto"])
    ap.add_argument("--plain", action="store_true", help="all fusions off + torch.optim.SGD")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--deterministic", action="store_true", help="MIOpen deterministic algorithms (slow)")
    ap.add_argument("--headline", action="store_true",
                    help="bench.py's config: batch 256, bf16 wire, auto shadow, 60 steps")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    if a.headline:
        a.batch, a.codec, a.bf16_weights, a.steps = 256, "bf16", "auto", max(a.steps, 60)
    return a


def _val(v):
    for t in (int, float):
        try:
            return t(v)
        except ValueError:
            pass
    return {"true": True, "false": False}.get(v.lower(), v)


def _cfg(spec):
    run, *mods = spec.split("+")
    d = _base_cfg(run)
    for m in mods:
        k, v = m.split("=", 1)
        d[k] = _val(v)
    return d


def _base_cfg(run):
    if run == "local":
        return {"mode": "local"}
    if run.startswith("async_md"):
        return {"mode": "ps_async", "max_delay": int(run[len("async_md"):])}
    if run == "async":
        return {"mode": "ps_async", "max_delay": -1}
    if run == "async_la":
        return {"mode": "ps_async", "max_delay": -1, "stale_lookahead": -1.0}
    if run == "async_model":
        return {"mode": "ps_async", "max_delay": -1, "ps_granularity": "model"}
    if run == "async_model_la":
        return {"mode": "ps_async", "max_delay": -1, "ps_granularity": "model", "stale_lookahead": -1.0}
    if run == "async_bucket":
        return {"mode": "ps_async", "max_delay": -1, "ps_granularity": "bucket", "bucket_mb": 16.0}
    if run == "async_slr":
        return {"mode": "ps_async", "max_delay": -1, "staleness_lr": True}
    if run == "async_prefetch":
        return {"mode": "ps_async", "max_delay": -1, "pull": "prefetch"}
    if run == "async_mc":
        return {"mode": "ps_async", "max_delay": -1, "stale_momentum": "comp"}
    raise ValueError(run)


def main(argv=None):
    a = parse(argv)
    if a.plain:
        os.environ.update(PLAIN_ENV)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.nn.functional as F

    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = a.deterministic
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from hipps.models import build_model

    g = torch.Generator(device="cpu").manual_seed(1000 + a.seed)
    x = torch.randn(a.batch, 3, a.image, a.image, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, a.classes, (a.batch,), generator=g).to(dev)
    recs = []
    for run in (["plain"] if a.plain else a.runs.split(",")):
        torch.manual_seed(a.seed)
        kw = {"num_classes": a.classes} if a.model.startswith("resnet") else {}
        model = build_model(a.model, **kw).to(dev).to(memory_format=torch.channels_last)
        stats = {}
        if run == "plain":
            opt = torch.optim.SGD(model.parameters(), lr=a.lr, momentum=a.momentum, weight_decay=a.wd)
        else:
            import hipps

            kw = dict(lr=a.lr, momentum=a.momentum, weight_decay=a.wd, code=a.codec, average=True,
                      bf16_weights=a.bf16_weights)
            kw.update(_cfg(run))
            opt = hipps.SGD(model.named_parameters(), **kw)
        losses, stale = [], []
        t0 = time.time()
        for s in range(a.steps):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(model(x), y)
            loss.backward()
            r = opt.step()
            data = r[1] if isinstance(r, tuple) else {}
            losses.append(float(loss.float().item()))
            if data and "staleness" in data:
                stale.append(float(data["staleness"]))
            if s % 10 == 0:
                print(f"[trajectory] {run} step {s} loss {losses[-1]:.4f}", file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        if hasattr(opt, "close"):
            eng = opt.engine
            opt.close()
            if hasattr(eng, "ps_stats"):
                stats = eng.ps_stats()
                stats.update(eng.transport_info())
        flat = torch.cat([p.detach().float().reshape(-1).cpu() for p in model.parameters()])
        recs.append({"variant": run, "model": a.model, "batch": a.batch, "image": a.image, "steps": a.steps,
                     "lr": a.lr, "losses": losses, "param_sha": hashlib.sha1(flat.numpy().tobytes()).hexdigest()[:16],
                     "param_norm": float(flat.norm()), "seconds": round(time.time() - t0, 2), "ps": stats,
                     "staleness": stale, "codec": a.codec, "bf16_weights": a.bf16_weights})
        print(json.dumps(recs[-1]), flush=True)
        del opt, model
    if a.out:
        with open(a.out, "w") as f:
            json.dump(recs, f)


if __name__ == "__main__":
    main()
