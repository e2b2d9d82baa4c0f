"""Probe the 1x1-conv MFMA GEMM core (hipps/csrc/gemm.hip k_conv1x1_nt) on plain [M, K] x [N, K]^T
problems: TFLOP/s per shape, with and without the BN-statistics epilogue, against a torch.matmul
(hipBLASLt) reference of the same product.

    python tools/gemm_probe.py                      # the shape table
    python tools/gemm_probe.py --shape 50176,1024,512 --iters 50   # one shape (for rocprofv3 --pmc)
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipps.ops._native import native  # noqa: E402

SHAPES = [  # (M, K, N): ResNet-50 bs256 1x1 GEMMs, then large steady-state problems
    (802816, 64, 256), (802816, 256, 64), (200704, 512, 128), (200704, 128, 512), (50176, 1024, 256),
    (50176, 256, 1024), (50176, 1024, 512), (12544, 2048, 512), (12544, 512, 2048),
    (65536, 4096, 4096), (32768, 2048, 2048)]


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


def run(M, K, N, it, stats=True, ref=True):
    C = native()
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    mt = C.conv1x1_mtiles(M)
    part = torch.empty(2, N, mt, device="cuda")
    t = timeit(lambda: C.conv1x1_forward(x, w, y, None, M, 1, 1), it)
    ts = timeit(lambda: C.conv1x1_forward(x, w, y, part, M, 1, 1), it) if stats else None
    tr = timeit(lambda: torch.matmul(x, w.t()), it) if ref else None
    r = torch.matmul(x[:4096].float(), w.float().t())
    C.conv1x1_forward(x, w, y, None, M, 1, 1)
    err = ((y[:4096].float() - r).abs().max() / r.abs().max()).item()
    fl = 2.0 * M * K * N
    return {"M": M, "K": K, "N": N, "ms": round(t, 4), "TFLOPs": round(fl / t / 1e9, 1),
            "stats_ms": None if ts is None else round(ts, 4),
            "hipblaslt_ms": None if tr is None else round(tr, 4),
            "hipblaslt_TFLOPs": None if tr is None else round(fl / tr / 1e9, 1),
            "TBps": round(2.0 * (M * K + M * N + N * K) / t / 1e9, 2), "rel_err": round(err, 5)}


CONV_SHAPES = [  # (M, Cin, Cout) of the stride-1 ResNet-50 bs256 1x1 convolutions
    (802816, 64, 64), (802816, 64, 256), (802816, 256, 64), (802816, 256, 128), (200704, 128, 512),
    (200704, 512, 128), (200704, 512, 256), (50176, 256, 1024), (50176, 1024, 256), (50176, 1024, 512),
    (12544, 512, 2048), (12544, 2048, 512)]


def run_wgrad(M, cin, cout, it):
    """weight gradient dW[Cout, Cin] = dy^T x: hipps k_conv1x1_wgrad2 vs hipBLASLt (fp32 out)."""
    C = native()
    x = (torch.randn(M, cin, device="cuda") * 0.5).to(torch.bfloat16)
    dy = (torch.randn(M, cout, device="cuda") * 0.5).to(torch.bfloat16)
    dw = torch.empty(cout, cin, device="cuda")
    t = timeit(lambda: C.conv1x1_wgrad(dy, x, dw, M, 1, 1, None, None), it)
    tr = timeit(lambda: torch.ops.aten.mm.dtype(dy.t(), x, torch.float32), it)
    tb = timeit(lambda: torch.mm(dy.t(), x), it)
    ref = torch.ops.aten.mm.dtype(dy.t(), x, torch.float32)
    C.conv1x1_wgrad(dy, x, dw, M, 1, 1, None, None)
    err = ((dw - ref).abs().max() / ref.abs().max()).item()
    fl = 2.0 * M * cin * cout
    return {"wgrad": [M, cin, cout], "hipps_ms": round(t, 4), "hipps_TFLOPs": round(fl / t / 1e9, 1),
            "hipblaslt_f32out_ms": round(tr, 4), "hipblaslt_bf16out_ms": round(tb, 4),
            "hipblaslt_TFLOPs": round(fl / min(tr, tb) / 1e9, 1), "rel_err": round(err, 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default=None, help="M,K,N: one shape, core kernel only")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.shape:
        M, K, N = (int(v) for v in a.shape.split(","))
        print(json.dumps(run(M, K, N, a.iters, stats=False, ref=False)), flush=True)
        return
    rows = []
    for M, cin, cout in CONV_SHAPES:
        r = run_wgrad(M, cin, cout, a.iters)
        rows.append(r)
        print(json.dumps(r), flush=True)
    for M, K, N in SHAPES:
        r = run(M, K, N, a.iters)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
