"""MIOpen 1x1 conv vs hipBLASLt GEMM (channels-last view) for ResNet-50 1x1 shapes, fwd+bwd, bf16."""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.backends.cudnn.benchmark = True

# (N, Cin, H, W, Cout) for the bottleneck 1x1 convs (stride 1) at bs256
SHAPES = [(256, 64, 56, 56, 64), (256, 64, 56, 56, 256), (256, 256, 56, 56, 64), (256, 256, 56, 56, 128),
          (256, 128, 28, 28, 512), (256, 512, 28, 28, 128), (256, 512, 28, 28, 256), (256, 256, 14, 14, 1024),
          (256, 1024, 14, 14, 256), (256, 1024, 14, 14, 512), (256, 512, 7, 7, 2048), (256, 2048, 7, 7, 512)]


def timeit(fn, it=20):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


class GemmConv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):  # x NHWC-contiguous [N,C,H,W] channels_last, w [Co, Ci, 1, 1]
        N, C, H, W = x.shape
        x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
        w2 = w.view(w.shape[0], C)
        y2 = x2 @ w2.t()
        ctx.save_for_backward(x2, w2)
        ctx.shape = (N, H, W)
        return y2.view(N, H, W, -1).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x2, w2 = ctx.saved_tensors
        N, H, W = ctx.shape
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, dy.shape[1])
        dx = (dy2 @ w2).view(N, H, W, -1).permute(0, 3, 1, 2)
        dw = (dy2.t() @ x2).view(w2.shape[0], w2.shape[1], 1, 1)
        return dx, dw


tot = {"miopen": 0.0, "gemm": 0.0}
rows = []
for N, Ci, H, W, Co in SHAPES:
    x = torch.randn(N, Ci, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(Co, Ci, 1, 1, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(N, Co, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)

    def conv():
        y = F.conv2d(xr, wr)
        y.backward(g)

    def gemm():
        y = GemmConv1x1.apply(xr, wr)
        y.backward(g)

    # correctness
    y1 = F.conv2d(x.float(), w.float())
    y2 = GemmConv1x1.apply(x, w).float()
    err = ((y1 - y2).abs().max() / y1.abs().max()).item()
    tc, tg = timeit(conv), timeit(gemm)
    fl = 3 * 2 * N * H * W * Ci * Co
    r = {"shape": [N, Ci, H, W, Co], "miopen_ms": round(tc, 3), "gemm_ms": round(tg, 3),
         "miopen_TF": round(fl / tc / 1e9, 1), "gemm_TF": round(fl / tg / 1e9, 1), "relerr": err}
    tot["miopen"] += tc
    tot["gemm"] += tg
    rows.append(r)
    print(json.dumps(r), flush=True)
print(json.dumps({"total_ms": tot}))
json.dump(rows, open(os.path.join(ROOT, "gpurun_out/conv1x1.json"), "w"), indent=1)
