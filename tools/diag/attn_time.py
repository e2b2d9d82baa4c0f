"""Time hipps flash attention (csrc/attn.hip) against PyTorch SDPA (aotriton on ROCm) on the
transformer configs' attention shapes, forward and backward, same process, interleaved.

    python tools/diag/attn_time.py [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hipps.ops.nn as hnn  # noqa: E402

SHAPES = {
    # name: B, S, Hq, Hkv, D, causal
    "bert-base b32": (32, 512, 12, 12, 64, False),
    "bert-base b256": (256, 512, 12, 12, 64, False),
    "llama3-1b b4": (4, 2048, 32, 8, 64, True),
    "llama3-8b b1": (1, 2048, 32, 8, 128, True),
}


def _time(fn, n=10):
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
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[n // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    out = {}
    for name, (B, S, Hq, Hkv, D, causal) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        torch.manual_seed(0)
        q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        g = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
        flops_f = 4.0 * B * Hq * S * S * D * (0.5 if causal else 1.0)
        flops_b = 2.5 * flops_f

        def ours_f():
            return hnn.attention(q, k, v, causal=causal)

        def sdpa_f():
            return F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                                  is_causal=causal, enable_gqa=Hq != Hkv).transpose(1, 2)

        row = {}
        for tag, f in (("hipps", ours_f), ("sdpa", sdpa_f)):
            with torch.no_grad():
                tf = _time(f)
            o = f()
            tb = _time(lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True))
            row[tag] = {"fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
                        "fwd_tflops": round(flops_f / tf / 1e9, 1), "bwd_tflops": round(flops_b / tb / 1e9, 1)}
        out[name] = row
        print(f"{name:16s} fwd hipps {row['hipps']['fwd_ms']:.3f} ms ({row['hipps']['fwd_tflops']} TF) "
              f"sdpa {row['sdpa']['fwd_ms']:.3f} ({row['sdpa']['fwd_tflops']}) | bwd hipps "
              f"{row['hipps']['bwd_ms']:.3f} ({row['hipps']['bwd_tflops']}) sdpa {row['sdpa']['bwd_ms']:.3f} "
              f"({row['sdpa']['bwd_tflops']})", flush=True)
        del q, k, v, g
        torch.cuda.empty_cache()
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
