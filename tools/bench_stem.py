"""Stem 7x7/s2 convolution: hipps' MFMA stem kernels (csrc/stem.hip) vs MIOpen, and MIOpen with
the 3 input channels zero-padded to 4 or 8.

Cin = 3 gives a 147-long reduction that MIOpen's implicit-GEMM solvers tile poorly. The padded
channels are zero, so the outputs are unchanged and the weight gradient of the real channels is the same.
    python tools/bench_stem.py [--batch 256]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    torch.manual_seed(0)
    n = args.batch
    cl = torch.channels_last
    x3 = torch.randn(n, 3, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    w3 = torch.randn(64, 3, 7, 7, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    y_ref = torch.ops.aten.convolution(x3, w3, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1)
    dy = torch.randn_like(y_ref)
    out = {}
    for c in (3, 4, 8):
        x = torch.zeros(n, c, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        x[:, :3] = x3
        w = torch.zeros(64, c, 7, 7, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        w[:, :3] = w3
        fwd = lambda: torch.ops.aten.convolution(x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1)
        wgr = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                          [False, True, False])[1]
        pad = lambda: torch.empty(n, c, 224, 224, device="cuda", dtype=torch.bfloat16,
                                  memory_format=cl).zero_()[:, :3].copy_(x3)
        y = fwd()
        dw = wgr()
        err = (y.float() - y_ref.float()).abs().max().item()
        out[f"c{c}"] = {"fwd_us": timeit(fwd), "wgrad_us": timeit(wgr), "pad_us": timeit(pad) if c > 3 else 0.0,
                        "max_abs_diff_vs_c3": err, "dw_shape": list(dw.shape)}
        print(f"C={c}", json.dumps(out[f"c{c}"]), flush=True)
    from hipps.ops._native import native

    w3c = w3.contiguous(memory_format=cl)
    y = torch.empty_like(y_ref)
    part = torch.empty(2, 64, native().stem_mtiles(n, y_ref.shape[2]), device="cuda")
    dw = torch.empty(64, 3, 7, 7, device="cuda").contiguous(memory_format=cl)
    native().stem_forward(x3, w3c, y, part)
    native().stem_wgrad(dy, x3, dw)
    ref_dw = torch.ops.aten.convolution_backward(dy, x3, w3, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                 [False, True, False])[1].float()
    out["hipps"] = {"fwd_us": timeit(lambda: native().stem_forward(x3, w3c, y, part)),
                    "wgrad_us": timeit(lambda: native().stem_wgrad(dy, x3, dw)),
                    "max_abs_diff_fwd_vs_miopen": (y.float() - y_ref.float()).abs().max().item(),
                    "max_rel_diff_wgrad_vs_miopen": ((dw - ref_dw).abs().max() / ref_dw.abs().max()).item()}
    print("hipps", json.dumps(out["hipps"]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
