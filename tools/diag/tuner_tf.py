"""Every kernel-tuner decision of a transformer step with each candidate's time (ms): which GEMM
shapes run on hipBLASLt and which on the gemm2 cores, and by how much.

    python tools/diag/tuner_tf.py --model bert-base --batch 32 --seq 512 [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import hipps
    from hipps.models.transformer import build
    from hipps.ops import nn as hnn

    torch.manual_seed(0)
    m = build(a.model).cuda()
    opt = hipps.SGD(m.named_parameters(), lr=1e-4, momentum=0.9, mode="ps_async", code="bf16", average=True, max_delay=0)
    vocab = m.c.vocab
    ids = torch.randint(0, vocab, (a.batch, a.seq), device="cuda")
    for _ in range(2):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(ids, ids)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    rows = []
    for key, times in hnn.TUNER.times.items():
        pick = hnn.TUNER.cache.get(key)
        best = min(times.values())
        rows.append({"key": [str(k) for k in key], "pick": pick,
                     "times_ms": {n: round(t, 4) for n, t in sorted(times.items(), key=lambda kv: kv[1])},
                     "blas_vs_pick": round(times.get("blas", times.get("mm", best)) / best, 3)})
    for r in rows:
        top = list(r["times_ms"].items())[:4]
        print(" ".join(r["key"]), "->", r["pick"], top, flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
    opt.close() if hasattr(opt, "close") else None


if __name__ == "__main__":
    main()
