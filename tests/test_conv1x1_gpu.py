"""GPU: MFMA 1x1-conv GEMM (hipps/csrc/gemm.hip) vs an fp32 PyTorch convolution, its fused BN
statistics epilogue, and the conv_bn autograd path vs the unfused modules."""
import pytest
import torch
import torch.nn.functional as F

from hipps.ops import nn as hnn
from hipps.ops._native import native

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [  # (images, Cin, H, W, Cout, stride)
    (2, 64, 56, 56, 256, 1),
    (2, 256, 56, 56, 64, 1),
    (3, 128, 7, 7, 64, 1),     # M = 147: partial last M tile
    (2, 256, 14, 14, 512, 2),  # strided (downsample) rows
    (1, 2048, 7, 7, 512, 1),
    (2, 512, 28, 28, 1024, 2),
    (8, 64, 9, 9, 128, 1),
]


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv1x1_matches_fp32_conv_and_stats(shape):
    n, cin, h, w, cout, s = shape
    torch.manual_seed(cin + cout)
    x = _cl(torch.randn(n, cin, h, w, device=DEV).to(torch.bfloat16))
    wt = (torch.randn(cout, cin, 1, 1, device=DEV) / cin ** 0.5).to(torch.bfloat16)
    ref = F.conv2d(x.float(), wt.float(), stride=s)
    y, part = hnn._Conv1x1.apply(x, wt, s)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, cout)  # stats are of the stored bf16 values
    mt = native().conv1x1_mtiles(yf.shape[0])
    assert part.shape == (2, cout, mt)
    torch.testing.assert_close(part[0].sum(1), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(1), (yf * yf).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("shape", SHAPES + [(2, 64, 5, 5, 64, 1), (1, 72, 7, 7, 136, 1)])
def test_conv1x1_wgrad_matches_fp32(shape):
    n, cin, h, w, cout, s = shape
    torch.manual_seed(7 + cin)
    x = _cl(torch.randn(n, cin, h, w, device=DEV).to(torch.bfloat16))
    ho = (h - 1) // s + 1
    dy = _cl(torch.randn(n, cout, ho, ho, device=DEV).to(torch.bfloat16))
    xs = x.float()[:, :, ::s, ::s]
    ref = torch.einsum("nchw,nkhw->kc", xs, dy.float())
    dw = torch.empty(cout, cin, device=DEV)
    native().conv1x1_wgrad(dy, x, dw, h, w, s)
    torch.testing.assert_close(dw, ref, rtol=2e-3, atol=2e-3 * (n * ho * ho) ** 0.5)


def test_conv1x1_exact_on_integers():
    """Small integers are exact in bf16 and fp32: any row/column/k mix-up shows up exactly."""
    n, cin, h, w, cout = 2, 128, 8, 8, 192
    g = torch.Generator(device="cpu").manual_seed(0)
    x = _cl(torch.randint(-3, 4, (n, cin, h, w), generator=g).float().to(DEV).to(torch.bfloat16))
    wt = torch.randint(-2, 3, (cout, cin, 1, 1), generator=g).float().to(DEV).to(torch.bfloat16)
    y, _ = hnn._Conv1x1.apply(x, wt, 1)
    assert torch.equal(y.float(), F.conv2d(x.float(), wt.float()))
    dy = _cl(torch.randint(-2, 3, y.shape, generator=g).float().to(DEV).to(torch.bfloat16))
    dw = torch.empty(cout, cin, device=DEV)
    native().conv1x1_wgrad(dy, x, dw, h, w, 1)
    assert torch.equal(dw, torch.einsum("nchw,nkhw->kc", x.float(), dy.float()))


@pytest.mark.parametrize("residual", [False, True])
@pytest.mark.parametrize("stride", [1, 2])
def test_conv_bn_autograd_matches_unfused(residual, stride):
    torch.manual_seed(1)
    cin, cout = 128, 256
    conv = torch.nn.Conv2d(cin, cout, 1, stride=stride, bias=False).to(DEV).to(memory_format=torch.channels_last)
    bn_a = hnn.FusedBatchNorm2d(cout, relu=True).to(DEV)
    bn_b = hnn.FusedBatchNorm2d(cout, relu=True).to(DEV)
    bn_b.load_state_dict(bn_a.state_dict())
    x0 = _cl(torch.randn(4, cin, 14, 14, device=DEV).to(torch.bfloat16))
    ho = (14 - 1) // stride + 1
    res = _cl(torch.randn(4, cout, ho, ho, device=DEV).to(torch.bfloat16)) if residual else None
    g = _cl(torch.randn(4, cout, ho, ho, device=DEV).to(torch.bfloat16))
    outs = []
    for fuse, bn in ((True, bn_a), (False, bn_b)):
        conv.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = hnn.conv_bn(conv, bn, x, residual=res, fuse=fuse)
        y.backward(g)
        outs.append((y.float(), x.grad.float(), conv.weight.grad.clone(), bn.weight.grad.clone(),
                     bn.running_mean.clone(), bn.running_var.clone()))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2)


def test_resnet50_fused_conv_matches_unfused():
    import hipps.models.resnet as R

    torch.manual_seed(0)
    m = R.resnet50(num_classes=10).to(DEV).to(memory_format=torch.channels_last)
    x = _cl(torch.randn(4, 3, 64, 64, device=DEV))
    out = {}
    for flag in (True, False):
        R._FUSED_CONV = flag
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().sum().backward()
        out[flag] = (y.float(), m.conv1.weight.grad.clone(), m.layer1[0].conv1.weight.grad.clone())
    R._FUSED_CONV = True
    for a, b in zip(out[True], out[False]):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2)
