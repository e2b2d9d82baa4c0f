"""GPU: ResNet stem kernels (hipps/csrc/stem.hip, 7x7/s2/p3, 3 -> 64 channels) vs an fp32 PyTorch
convolution: forward, the BatchNorm partial statistics of its epilogue, the weight gradient, and the
ResNet-50 stem routed through them (with the MIOpen path as the A/B reference)."""
import pytest
import torch
import torch.nn.functional as F

from hipps.ops import nn as hnn
from hipps.ops._native import native

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [  # (images, H, W)
    (2, 224, 224),  # ResNet-50: 112x112 outputs, 14 row groups of 8
    (3, 56, 40),    # 28x20 outputs: partial 16-pixel fragments, row groups past Ho
    (1, 37, 16),    # odd height, 19x8 outputs
    (2, 64, 256),   # 128-wide outputs (the widest staged dy row)
]


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _inputs(n, h, w, seed):
    torch.manual_seed(seed)
    x = _cl(torch.randn(n, 3, h, w, device=DEV).to(torch.bfloat16))
    wt = _cl((torch.randn(64, 3, 7, 7, device=DEV) / 147 ** 0.5).to(torch.bfloat16))
    return x, wt


@pytest.mark.parametrize("shape", SHAPES)
def test_stem_forward_matches_fp32_conv_and_stats(shape):
    n, h, w = shape
    x, wt = _inputs(n, h, w, h + w)
    ref = F.conv2d(x.float(), wt.float(), stride=2, padding=3)
    y = _cl(torch.empty(ref.shape, device=DEV, dtype=torch.bfloat16))
    mt = native().stem_mtiles(n, ref.shape[2])
    part = torch.empty(2, 64, mt, device=DEV)
    native().stem_forward(x, wt, y, part)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)  # statistics of the stored bf16 values
    torch.testing.assert_close(part[0].sum(1), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(1), (yf * yf).sum(0), rtol=1e-4, atol=1e-2)
    y2 = _cl(torch.empty_like(y))
    native().stem_forward(x, wt, y2)  # no statistics: same outputs
    assert torch.equal(y, y2)


@pytest.mark.parametrize("shape", SHAPES)
def test_stem_wgrad_matches_fp32(shape):
    n, h, w = shape
    x, wt = _inputs(n, h, w, 3 * h + w)
    xf = x.float().requires_grad_(False)
    wf = wt.float().requires_grad_(True)
    ref_y = F.conv2d(xf, wf, stride=2, padding=3)
    dy = _cl(torch.randn(ref_y.shape, device=DEV).to(torch.bfloat16))
    (ref_y * dy.float()).sum().backward()
    dw = _cl(torch.empty(64, 3, 7, 7, device=DEV))
    native().stem_wgrad(dy, x, dw)
    m = n * ref_y.shape[2] * ref_y.shape[3]
    torch.testing.assert_close(dw, wf.grad, rtol=2e-3, atol=2e-3 * m ** 0.5)
    dw2 = _cl(torch.empty_like(dw))
    native().stem_wgrad(dy, x, dw2)
    assert torch.equal(dw, dw2)  # fixed-order slab sum: bitwise repeatable


def test_stem_nonfinite_input_stays_local():
    """A NaN input pixel may only reach the outputs whose window covers it (zero-weighted padding
    lanes of the k steps must not carry it into neighbouring pixels)."""
    x, wt = _inputs(1, 32, 32, 5)
    x[0, 1, 10, 10] = float("nan")
    y = _cl(torch.empty(1, 64, 16, 16, device=DEV, dtype=torch.bfloat16))
    native().stem_forward(x, wt, y)
    bad = torch.isnan(y.float()).any(1)[0]
    # input (10, 10) is in the windows of outputs ho, wo with |2*ho - 10| <= 3: ho, wo in {4, 5, 6}
    expect = torch.zeros(16, 16, dtype=torch.bool, device=DEV)
    expect[4:7, 4:7] = True
    assert torch.equal(bad, expect)


def test_resnet_stem_routes_through_hipps_and_matches_miopen():
    from hipps.models import resnet50

    torch.manual_seed(0)
    m = resnet50().to(DEV).to(memory_format=torch.channels_last)
    x = _cl(torch.randn(4, 3, 224, 224, device=DEV))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert hnn.stem_ok(m.conv1, x)
        y, part = hnn.conv2d_stats(m.conv1, x)
    assert part is not None and part.shape[1] == 64  # only the hipps stem returns statistics
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = m.conv1(x)
    torch.testing.assert_close(y.float(), ref.float(), rtol=2e-2, atol=2e-2)
    # weight gradient through autograd into the fp32 master
    dy = torch.randn_like(ref.float())
    (y.float() * dy).sum().backward()
    g_own = m.conv1.weight.grad.clone()
    m.conv1.weight.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = m.conv1(x)
    (ref.float() * dy).sum().backward()
    assert g_own.dtype == torch.float32
    torch.testing.assert_close(g_own, m.conv1.weight.grad, rtol=2e-2, atol=2e-2 * g_own.abs().max().item())


@pytest.mark.parametrize("shape", [(4, 112, 112), (3, 27, 20)])
def test_bn_relu_pool_bit_identical_to_bn_then_pool(shape):
    """_BNReluPool (BN apply + ReLU in the pool's load) vs the fused BN module then the pool module:
    pooled values, running statistics and every gradient bitwise equal."""
    n, h, w = shape
    torch.manual_seed(h)
    y = _cl(torch.randn(n, 64, h, w, device=DEV).mul_(3).add_(0.5).to(torch.bfloat16))
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
    part = torch.stack([yf.sum(0), (yf * yf).sum(0)]).unsqueeze(-1).contiguous()  # one partial column
    outs = []
    for fused in (True, False):
        bn = hnn.FusedBatchNorm2d(64, relu=True).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(-1.5, 2.0, 64))  # negative scales too
            bn.bias.copy_(torch.linspace(-0.5, 0.5, 64))
        pool = hnn.MaxPool2d(3, stride=2, padding=1)
        yi = y.detach().clone().requires_grad_(True)
        out = hnn.bn_relu_maxpool(bn, pool, yi, part) if fused else pool(bn(yi, stats=part))
        g = _cl(torch.randn(out.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(1)).to(torch.bfloat16))
        out.backward(g)
        outs.append((out.detach(), yi.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("fused_bwd", [True, False])
def test_resnet_stem_route(fused_bwd, monkeypatch):
    """The ResNet stem runs _StemBlock (default, HIPPS_FUSED_STEMBWD=2 or 1) or _StemConv +
    _BNReluPool (HIPPS_FUSED_STEMBWD=0)."""
    from hipps.models import resnet as R
    from hipps.models import resnet50

    monkeypatch.setattr(R, "_FUSED_STEM_BWD", fused_bwd)
    m = resnet50().to(DEV).to(memory_format=torch.channels_last)
    x = _cl(torch.randn(2, 3, 64, 64, device=DEV))
    calls = []
    for cls in (hnn._StemBlock, hnn._BNReluPool):
        orig = cls.apply
        monkeypatch.setattr(cls, "apply", (lambda o, c: lambda *a: calls.append(c.__name__) or o(*a))(orig, cls))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        m(x).float().sum().backward()
    assert calls == (["_StemBlock"] if fused_bwd else ["_BNReluPool"])
    assert m.bn1.weight.grad is not None and torch.isfinite(m.conv1.weight.grad).all()


@pytest.mark.parametrize("quad", [True, False])
@pytest.mark.parametrize("materialize_dy", [False, True])
@pytest.mark.parametrize("n", [4, 2, 3])
def test_stem_block_matches_unfused_ops(n, materialize_dy, quad, monkeypatch):
    """_StemBlock (fused stem backward: BN reductions on a recomputed pool gradient, dy staged into
    the weight gradient -- or, materialize_dy (HIPPS_FUSED_STEMBWD=2), written by one elementwise
    pass and read by the plain weight gradient) vs _StemConv -> FusedBatchNorm2d -> MaxPool2d on the
    hipps kernels: identical forward and running statistics; gradients equal up to the BN
    reduction order."""
    monkeypatch.setattr(hnn, "_STEM_BWD_DY", materialize_dy)
    monkeypatch.setattr(hnn, "_STEM_QUAD", quad)
    torch.manual_seed(n)
    # n = 3: an odd number of stem output rows (98 x 72 -> 49 x 36; pooled 25 x 18), so the 2x2 blocks
    # of the quad kernels have missing pixels and missing windows at the edges
    hw = {4: (224, 224), 2: (96, 64), 3: (98, 72)}[n]
    x = _cl(torch.randn(n, 3, hw[0], hw[1], device=DEV).to(torch.bfloat16))
    res = []
    for fused in (True, False):
        torch.manual_seed(1)
        conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(DEV).to(memory_format=torch.channels_last)
        bn = hnn.FusedBatchNorm2d(64, relu=True).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(-1.5, 2.0, 64))
            bn.bias.copy_(torch.linspace(-0.5, 0.5, 64))
        pool = hnn.MaxPool2d(3, stride=2, padding=1)
        if fused:
            assert hnn.stem_block_ok(conv, bn, pool, x)
            out = hnn.stem_block(conv, bn, pool, x)
        else:
            y, part = hnn._StemConv.apply(x, conv.weight, True)
            out = pool(bn(y, stats=part))
        g = _cl(torch.randn(out.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(2)).to(torch.bfloat16))
        out.backward(g)
        res.append((out.detach(), bn.running_mean, bn.running_var, bn.weight.grad, bn.bias.grad, conv.weight.grad))
    (o1, rm1, rv1, bw1, bb1, cw1), (o2, rm2, rv2, bw2, bb2, cw2) = res
    assert torch.equal(o1, o2) and torch.equal(rm1, rm2) and torch.equal(rv1, rv2)
    torch.testing.assert_close(bw1, bw2, rtol=1e-4, atol=1e-4 * bw2.abs().max().item())
    torch.testing.assert_close(bb1, bb2, rtol=1e-4, atol=1e-4 * bb2.abs().max().item())
    torch.testing.assert_close(cw1, cw2, rtol=2e-3, atol=2e-3 * cw2.abs().max().item())
