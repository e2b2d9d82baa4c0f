#!/usr/bin/env python3
"""Probe the second-generation conv GEMM core (hipps/csrc/gemm2.hip) against the first core
(gemm.hip k_conv1x1_nt / convkxk_forward) and the vendor libraries (hipBLASLt via torch.matmul,
MIOpen via F.conv2d), per ResNet-50 bs256 shape and per block tile; checks every result against
an fp32 reference first.

    python tools/gemm2_probe.py --out gpurun_out/g2/probe.json
    python tools/gemm2_probe.py --only 50176,1024,512 --iters 50       # one GEMM (for rocprofv3)
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops._native import native  # noqa: E402

GEMMS = [  # (M, K, N): ResNet-50 bs256 1x1 convolutions + large steady-state problems
    (802816, 64, 256), (802816, 256, 64), (200704, 512, 128), (200704, 128, 512), (50176, 1024, 256),
    (50176, 256, 1024), (50176, 1024, 512), (12544, 2048, 512), (12544, 512, 2048),
    (65536, 4096, 4096), (32768, 2048, 2048)]
CONVS = [  # (Cin, H, Cout, stride): ResNet-50 bs256 3x3 convolutions (pad 1)
    (64, 56, 64, 1), (128, 56, 128, 2), (128, 28, 128, 1), (256, 28, 256, 2), (256, 14, 256, 1),
    (512, 14, 512, 2), (512, 7, 512, 1)]
TILES = [(256, 256, 2), (256, 256, 5), (256, 256, 6), (256, 128, 2), (256, 128, 3), (128, 128, 2), (256, 64, 2), (128, 64, 2),
         (128, 64, 3)]  # (bm, bn, LDS stages; 4 = k-half units, 5 = ping-pong wave groups, 6 = 32x32x16 MFMA)


def timeit(fn, it):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def gemm_row(M, K, N, it):
    C = native()
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    ref = (x[:4096].float() @ w.float().t())
    row = {"M": M, "K": K, "N": N}
    flop = 2.0 * M * N * K
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for bm, bn, ns in TILES:
        if N % bn:
            continue
        y.zero_()
        C.gemm2_conv(x, w, y, None, None, None, M, 1, bm=bm, bn=bn, stages=ns)
        torch.cuda.synchronize()
        err = rel_err(y[:4096], ref)
        assert err < 2e-2, (M, K, N, bm, bn, err)
        ms = timeit(lambda: C.gemm2_conv(x, w, y, None, None, None, M, 1, bm=bm, bn=bn, stages=ns), it)
        row[f"g2_{bm}x{bn}s{ns}_ms"] = round(ms, 4)
        row[f"g2_{bm}x{bn}s{ns}_TF"] = round(flop / ms / 1e9, 1)
    mt = C.gemm2_mtiles(M, N, K, 0)
    part = torch.empty(2, N, mt, device="cuda")
    ms = timeit(lambda: C.gemm2_conv(x, w, y, part, None, None, M, 1), it)
    row["g2_auto_stats_ms"] = round(ms, 4)
    y1 = torch.empty_like(y)
    ms1 = timeit(lambda: C.conv1x1_forward(x, w, y1, None, M, 1, 1, None, None, None, None, None, None, None, None,
                                           None, None), it)
    row["g1_ms"] = round(ms1, 4)
    row["g1_TF"] = round(flop / ms1 / 1e9, 1)
    msb = timeit(lambda: torch.matmul(x, w.t()), it)
    row["hipblaslt_ms"] = round(msb, 4)
    row["hipblaslt_TF"] = round(flop / msb / 1e9, 1)
    best = min((v, k) for k, v in row.items() if k.startswith("g2_") and k.endswith("_ms") and "stats" not in k)
    row["g2_best"] = best[1]
    row["g2_best_TF"] = round(flop / best[0] / 1e9, 1)
    return row


def conv_row(cin, h, cout, st, it):
    C = native()
    cl = torch.channels_last
    x = torch.randn(256, cin, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    ho = (h + 2 - 3) // st + 1
    M = 256 * ho * ho
    flop = 2.0 * M * cout * 9 * cin
    ref = F.conv2d(x[:4].float(), w.float(), stride=st, padding=1)
    row = {"Cin": cin, "H": h, "Cout": cout, "stride": st, "M": M}
    y = torch.empty(256, cout, ho, ho, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    for bm, bn, ns in TILES:
        if cout % bn:
            continue
        y.zero_()
        C.gemm2_conv(x, w, y, None, None, None, h, h, st, 3, 3, 1, bm, bn, stages=ns)
        torch.cuda.synchronize()
        err = rel_err(y[:4], ref)
        assert err < 2e-2, (cin, h, cout, st, bm, bn, err)
        ms = timeit(lambda: C.gemm2_conv(x, w, y, None, None, None, h, h, st, 3, 3, 1, bm, bn, stages=ns), it)
        row[f"g2_{bm}x{bn}s{ns}_ms"] = round(ms, 4)
        row[f"g2_{bm}x{bn}s{ns}_TF"] = round(flop / ms / 1e9, 1)
    y1 = torch.empty_like(y)
    ms1 = timeit(lambda: C.convkxk_forward(x, w, y1, None, st, 1), it)
    row["g1_ms"] = round(ms1, 4)
    torch.backends.cudnn.benchmark = True
    msm = timeit(lambda: F.conv2d(x, w, stride=st, padding=1), it)
    row["miopen_find_ms"] = round(msm, 4)
    row["miopen_TF"] = round(flop / msm / 1e9, 1)
    best = min((v, k) for k, v in row.items() if k.startswith("g2_") and k.endswith("_ms"))
    row["g2_best"] = best[1]
    row["g2_best_TF"] = round(flop / best[0] / 1e9, 1)
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None, help="M,K,N: one GEMM, auto tile, --iters launches")
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-convs", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(0)
    if a.only:
        M, K, N = (int(v) for v in a.only.split(","))
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(a.iters):
            native().gemm2_conv(x, w, y, None, None, None, M, 1)
        torch.cuda.synchronize()
        return
    rows = []
    for M, K, N in GEMMS:
        rows.append(gemm_row(M, K, N, a.iters))
        print(json.dumps(rows[-1]), flush=True)
    if not a.no_convs:
        for cin, h, cout, st in CONVS:
            rows.append(conv_row(cin, h, cout, st, a.iters))
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
