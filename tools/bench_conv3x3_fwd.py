"""Microbenchmark: ResNet-50 3x3 convolution forward (bs 256, channels-last bf16), MIOpen/CK
(aten.convolution) vs hipps convkxk_forward (implicit-GEMM MFMA, optional BN-stats epilogue)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops._native import native  # noqa: E402

# (channels, input size, stride) of the 16 3x3 convs (x count)
SHAPES = [(64, 56, 1, 3), (128, 56, 2, 1), (128, 28, 1, 3), (256, 28, 2, 1), (256, 14, 1, 5), (512, 14, 2, 1),
          (512, 7, 1, 2)]
B = int(os.environ.get("BATCH", "256"))
# MIOpen as the ResNet bench runs it: Find over all solvers (cudnn.benchmark), not the immediate-mode pick
torch.backends.cudnn.benchmark = os.environ.get("FIND", "1") != "0"


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


rows, tot = [], {"miopen_ms": 0.0, "hipps_ms": 0.0, "hipps_stats_ms": 0.0}
for c, h, st, cnt in SHAPES:
    x = torch.randn(B, c, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda") / (3 * c ** 0.5)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution(x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1)
    y = torch.empty_like(ref, memory_format=torch.channels_last)
    ho = ref.shape[2]
    part = torch.empty(2, c, native().conv1x1_mtiles(B * ho * ho), device="cuda")
    t_mi = timeit(lambda: torch.ops.aten.convolution(x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1))
    t_h = timeit(lambda: native().convkxk_forward(x, w, y, None, st, 1))
    t_hs = timeit(lambda: native().convkxk_forward(x, w, y, part, st, 1))
    native().convkxk_forward(x, w, y, part, st, 1)
    torch.cuda.synchronize()
    err = float((y.float() - ref.float()).norm() / ref.float().norm())
    s_ref = y.float().sum((0, 2, 3))
    s_err = float((part[0].sum(1) - s_ref).abs().max() / s_ref.abs().max().clamp_min(1e-6))
    flops = 2 * B * ho * ho * c * c * 9
    row = {"c": c, "hw": h, "stride": st, "count": cnt, "miopen_ms": round(t_mi, 4), "hipps_ms": round(t_h, 4),
           "hipps_stats_ms": round(t_hs, 4), "hipps_TFLOPs": round(flops / t_h / 1e9, 1),
           "miopen_TFLOPs": round(flops / t_mi / 1e9, 1), "rel_err": round(err, 5), "stats_err": round(s_err, 6)}
    rows.append(row)
    for k in tot:
        tot[k] += row[k] * cnt
    print(json.dumps(row), flush=True)
print(json.dumps({"per_step_fwd_ms": {k: round(v, 3) for k, v in tot.items()}}))
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump({"rows": rows, "total": tot}, f, indent=1)
