"""Microbenchmark: ResNet-50 1x1 convolutions (bs 256, channels-last bf16), forward.

  miopen        F.conv2d (MIOpen)                        -> y
  miopen+stats  F.conv2d + the fused-BN statistics pass  (what the unfused path pays)
  hipps         MFMA GEMM with BN statistics in the epilogue (hipps/csrc/gemm.hip)
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops import nn as hnn  # noqa: E402
from hipps.ops._native import native  # noqa: E402

SHAPES = [  # (Cin, H, Cout, stride) at batch 256
    (64, 56, 64, 1), (64, 56, 256, 1), (256, 56, 64, 1), (256, 56, 128, 1), (256, 56, 512, 2),
    (128, 28, 512, 1), (512, 28, 128, 1), (512, 28, 256, 1), (512, 28, 1024, 2),
    (256, 14, 1024, 1), (1024, 14, 256, 1), (1024, 14, 512, 1), (1024, 14, 2048, 2),
    (512, 7, 2048, 1), (2048, 7, 512, 1)]


def timeit(fn, it=30):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


rows = []
for cin, h, cout, st in SHAPES:
    x = torch.randn(256, cin, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
    ho = (h - 1) // st + 1
    M = 256 * ho * ho
    y = torch.empty(256, cout, ho, ho, dtype=torch.bfloat16, device="cuda").contiguous(memory_format=torch.channels_last)
    mt = native().conv1x1_mtiles(M)
    part = torch.empty(2, cout, mt, device="cuda")
    f32 = dict(device="cuda", dtype=torch.float32)
    bw, bb = torch.ones(cout, **f32), torch.zeros(cout, **f32)
    rm, rv = torch.zeros(cout, **f32), torch.ones(cout, **f32)
    mean, inv, sc, sh = (torch.empty(cout, **f32) for _ in range(4))
    yb = torch.empty_like(y)

    t_mi = timeit(lambda: F.conv2d(x, w, stride=st))
    t_mi_bn = timeit(lambda: native().bn_forward_train(F.conv2d(x, w, stride=st), None, yb, bw, bb, rm, rv, mean, inv,
                                                       sc, sh, cout, 1e-5, 0.1, True, None))
    t_h = timeit(lambda: native().conv1x1_forward(x, w.view(cout, cin), y, part, h, h, st))
    t_h_bn = timeit(lambda: (native().conv1x1_forward(x, w.view(cout, cin), y, part, h, h, st),
                             native().bn_forward_partials(part, mt, y, None, yb, bw, bb, rm, rv, mean, inv, sc, sh,
                                                          cout, 1e-5, 0.1, True, None)))
    # backward input gradient (stride 1): MIOpen dgrad vs the same GEMM on the transposed weight
    t_mi_dg = t_h_dg = None
    if st == 1:
        dy = torch.randn_like(y)
        wt = w.view(cout, cin).t().contiguous()
        dx = torch.empty_like(x)
        t_mi_dg = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                     [0, 0], 1, [True, False, False]))
        t_h_dg = timeit(lambda: native().conv1x1_forward(dy, wt, dx, None, h, h, 1))
        ref_dx = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        dg_err = ((dx.float() - ref_dx.float()).abs().max() / ref_dx.float().abs().max()).item()
    dyw = torch.randn_like(y)
    dwo = torch.empty(cout, cin, device="cuda")
    t_mi_wg = timeit(lambda: torch.ops.aten.convolution_backward(dyw, x, w, None, [st, st], [0, 0], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]))
    t_h_wg = timeit(lambda: native().conv1x1_wgrad(dyw, x, dwo, h, h, st))
    ref_dw = torch.ops.aten.convolution_backward(dyw, x, w, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1,
                                                 [False, True, False])[1].float().view(cout, cin)
    wg_err = ((dwo - ref_dw).abs().max() / ref_dw.abs().max()).item()
    flops = 2.0 * M * cin * cout
    byts = (256 * cin * h * h + M * cout) * 2
    ref = F.conv2d(x, w, stride=st)
    err = ((y.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    r = {"cin": cin, "hw": h, "cout": cout, "stride": st, "miopen_ms": round(t_mi, 4), "hipps_ms": round(t_h, 4),
         "miopen_plus_bn_ms": round(t_mi_bn, 4), "hipps_plus_bn_ms": round(t_h_bn, 4),
         "hipps_TFLOPs": round(flops / t_h / 1e9, 1), "hipps_TBps": round(byts / t_h / 1e9, 2),
         "rel_err": round(err, 5),
         "miopen_dgrad_ms": None if t_mi_dg is None else round(t_mi_dg, 4),
         "hipps_dgrad_ms": None if t_h_dg is None else round(t_h_dg, 4),
         "dgrad_rel_err": None if t_h_dg is None else round(dg_err, 5),
         "miopen_wgrad_ms": round(t_mi_wg, 4), "hipps_wgrad_ms": round(t_h_wg, 4), "wgrad_rel_err": round(wg_err, 5)}
    rows.append(r)
    print(json.dumps(r), flush=True)
tot = {k: round(sum(r[k] or 0 for r in rows), 3) for k in ("miopen_ms", "hipps_ms", "miopen_plus_bn_ms",
                                                          "hipps_plus_bn_ms", "miopen_dgrad_ms", "hipps_dgrad_ms",
                                                          "miopen_wgrad_ms", "hipps_wgrad_ms")}
print(json.dumps({"total": tot}))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump({"rows": rows, "total": tot}, open(os.path.join(ROOT, "gpurun_out/bench_conv1x1.json"), "w"), indent=1)
