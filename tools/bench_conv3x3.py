"""Microbenchmark: ResNet-50 3x3 convolution weight gradients (bs 256, channels-last bf16):
MIOpen (aten.convolution_backward, weight only) vs hipps conv_wgrad (implicit-GEMM MFMA)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops._native import native  # noqa: E402

SHAPES = [(64, 56, 1), (128, 56, 2), (128, 28, 1), (256, 28, 2), (256, 14, 1), (512, 14, 2), (512, 7, 1)]
B = int(os.environ.get("BATCH", "256"))


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


tot = {"miopen_ms": 0.0, "hipps_ms": 0.0}
for c, h, st in SHAPES:
    x = torch.randn(B, c, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ho = (h + 2 - 3) // st + 1
    dy = torch.randn(B, c, ho, ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(c, c, 3, 3, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = torch.empty(c, c, 3, 3, device="cuda", memory_format=torch.channels_last)
    t_mi = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1,
                                                              [False, True, False]))
    t_h = timeit(lambda: native().conv_wgrad(dy, x, dw, 3, 3, st, 1))
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1].float()
    err = ((dw - ref).abs().max() / ref.abs().max()).item()
    fl = 2.0 * B * ho * ho * c * c * 9
    row = {"cin": c, "hw": h, "stride": st, "miopen_ms": round(t_mi, 4), "hipps_ms": round(t_h, 4),
           "hipps_TFLOPs": round(fl / t_h / 1e9, 1), "miopen_TFLOPs": round(fl / t_mi / 1e9, 1), "rel_err": round(err, 5)}
    tot["miopen_ms"] += t_mi
    tot["hipps_ms"] += t_h
    print(json.dumps(row), flush=True)
print(json.dumps({"total": {k: round(v, 3) for k, v in tot.items()}}))
