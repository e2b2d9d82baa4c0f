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
    # one partial column per M tile of whichever core the tuner picked (first core: 128 rows,
    # gemm2: 128 or 256)
    M = yf.shape[0]
    assert part.shape[:2] == (2, cout)
    assert part.shape[2] in (native().conv1x1_mtiles(M), native().gemm2_mtiles(M, cout, cin, 128),
                             native().gemm2_mtiles(M, cout, cin, 256))
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


KXK = [  # (images, Cin, H, W, Cout, k, stride, pad)
    (2, 64, 14, 14, 64, 3, 1, 1),
    (2, 128, 15, 13, 256, 3, 2, 1),   # odd sizes, stride 2: padding on one side only
    (4, 256, 7, 7, 128, 3, 1, 1),
    (1, 64, 9, 9, 128, 5, 1, 2),
    (2, 128, 6, 6, 64, 1, 1, 0),      # 1x1 through the general entry point
]


@pytest.mark.parametrize("shape", KXK)
def test_conv_wgrad_matches_fp32(shape):
    n, cin, h, w, cout, k, s, p = shape
    torch.manual_seed(11 + cin + k)
    x = _cl(torch.randn(n, cin, h, w, device=DEV).to(torch.bfloat16))
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    dy = _cl(torch.randn(n, cout, ho, wo, device=DEV).to(torch.bfloat16))
    wt = torch.zeros(cout, cin, k, k, device=DEV)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), wt, None, [s, s], [p, p], [1, 1], False, [0, 0],
                                              1, [False, True, False])[1]
    dw = torch.empty(cout, cin, k, k, device=DEV, memory_format=torch.channels_last)
    native().conv_wgrad(dy, x, dw, k, k, s, p)
    torch.testing.assert_close(dw, ref, rtol=2e-3, atol=2e-3 * (n * ho * wo) ** 0.5)


def test_conv3x3_autograd_matches_conv():
    torch.manual_seed(12)
    conv = torch.nn.Conv2d(128, 128, 3, stride=2, padding=1, bias=False).to(DEV).to(memory_format=torch.channels_last)
    x0 = _cl(torch.randn(4, 128, 14, 14, device=DEV).to(torch.bfloat16))
    outs = []
    for fuse in (True, False):
        conv.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = hnn.conv2d(conv, x, fuse=fuse)
        y.float().square().sum().backward()
        outs.append((y.float(), x.grad.float(), conv.weight.grad.float()))
    for a, b in zip(*outs):
        scale = b.abs().max().item() + 1e-6
        torch.testing.assert_close(a / scale, b / scale, rtol=0, atol=1e-2)


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


@pytest.mark.parametrize("masked", [False, True])
def test_conv1x1_epilogue_add(masked):
    """dgrad epilogue: y = conv(x) + add (* ReLU bits) vs the eager sum of the rounded conv."""
    torch.manual_seed(3)
    n, cin, h, w, cout = 2, 128, 9, 9, 256
    x = _cl(torch.randn(n, cin, h, w, device=DEV).to(torch.bfloat16))
    wt = (torch.randn(cout, cin, device=DEV) / cin ** 0.5).to(torch.bfloat16)
    add = _cl(torch.randn(n, cout, h, w, device=DEV).to(torch.bfloat16))
    mask = torch.randint(0, 256, (add.numel() // 8,), dtype=torch.uint8, device=DEV) if masked else None
    y0 = _cl(torch.empty(n, cout, h, w, device=DEV, dtype=torch.bfloat16))
    y1 = torch.empty_like(y0)
    native().conv1x1_forward(x, wt, y0, None, h, w, 1)
    native().conv1x1_forward(x, wt, y1, None, h, w, 1, add, mask)
    want = (y0.float() + hnn._masked(add, mask, cout).float()).to(torch.bfloat16)
    assert torch.equal(y1, want)


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (2, 16, 7, 9), (3, 8, 1, 2), (2, 32, 6, 6)])
def test_maxpool3s2_matches_torch(shape):
    torch.manual_seed(4)
    x0 = _cl(torch.randint(-3, 4, shape, device=DEV).to(torch.bfloat16))  # many ties: tie rule must match
    x = x0.clone().requires_grad_(True)
    xr = x0.float().clone().requires_grad_(True)
    pool = hnn.MaxPool2d(3, stride=2, padding=1)
    y = pool(x)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y.float(), yr)
    g = _cl(torch.randn(yr.shape, device=DEV).to(torch.bfloat16))
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


def _resnet_run(R, m, x, fused, bf16=True):
    """One forward/backward with every runtime fusion switch on or off: 1x1 MFMA conv + BN stats,
    residual-gradient and BN-backward epilogues, 3x3 weight gradient, own 1x1 weight gradient,
    3x3 input gradient as a forward conv, fused BN, stem max pool."""
    import hipps.ops.nn as N

    saved = (R._FUSED_CONV, R._FUSED_GRAD, R._FUSED_BNGRAD, R._FUSED_WGRAD, N._OWN_WGRAD, N._DGRAD_AS_FWD,
             N._OWN_KXK_FWD)
    bns = [mod for mod in m.modules() if isinstance(mod, N.FusedBatchNorm2d)]
    R._FUSED_CONV = R._FUSED_GRAD = R._FUSED_BNGRAD = R._FUSED_WGRAD = fused
    N._OWN_WGRAD = N._DGRAD_AS_FWD = N._OWN_KXK_FWD = fused
    m.maxpool.fused = fused
    for bn in bns:
        bn.fused = fused
    try:
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            y = m(x)
        y.float().sum().backward()
    finally:
        (R._FUSED_CONV, R._FUSED_GRAD, R._FUSED_BNGRAD, R._FUSED_WGRAD, N._OWN_WGRAD, N._DGRAD_AS_FWD,
         N._OWN_KXK_FWD) = saved
        m.maxpool.fused = True
        for bn in bns:
            bn.fused = True
    return (y.float(), m.conv1.weight.grad.clone(), m.bn1.weight.grad.clone(), m.layer1[0].conv1.weight.grad.clone(),
            m.layer1[1].conv1.weight.grad.clone(), m.layer1[1].conv2.weight.grad.clone(),
            m.layer2[0].downsample[0].weight.grad.clone(), m.layer3[2].conv2.weight.grad.clone(),
            m.layer4[2].bn3.weight.grad.clone())


def _rel(u, v):
    return float((u.float() - v.float()).norm() / v.float().norm().clamp_min(1e-12))


def test_resnet50_fused_conv_matches_unfused():
    """All ResNet fusions against the plain path (MIOpen convs, eager BN, autograd adds, PyTorch
    pool), both under bf16 autocast, judged against a plain fp32 run: the fused path may not add
    error beyond what bf16 itself costs (50 layers of bf16 with training-mode BN drift far from
    fp32, so a fixed tolerance between the two bf16 runs says little).  bn3 weights are drawn in
    [0.5, 1.5]: zero-init would make every residual branch gradient exactly zero in all runs."""
    import hipps.models.resnet as R

    torch.manual_seed(0)
    m = R.resnet50(num_classes=10).to(DEV).to(memory_format=torch.channels_last)
    for blk in [b for layer in (m.layer1, m.layer2, m.layer3, m.layer4) for b in layer]:
        torch.nn.init.uniform_(blk.bn3.weight, 0.5, 1.5)
    x = _cl(torch.randn(8, 3, 96, 96, device=DEV))
    fused = _resnet_run(R, m, x, True)
    plain = _resnet_run(R, m, x, False)
    ref = _resnet_run(R, m, x, False, bf16=False)
    names = ["out", "stem", "bn1.w", "l1.0.conv1", "l1.1.conv1", "l1.1.conv2", "l2.0.down", "l3.2.conv2", "l4.2.bn3.w"]
    for name, f, p, r in zip(names, fused, plain, ref):
        assert float(r.float().abs().max()) > 0, name  # every compared gradient is live
        ef, ep = _rel(f, r), _rel(p, r)
        assert ef <= 1.5 * ep + 0.02, (name, ef, ep)


@pytest.mark.parametrize("bngrad", [False, True])
def test_bottleneck_chain_bn_backward_in_epilogue(bngrad):
    """Two chained blocks (downsample, then identity): the second block's conv1 dgrad epilogue
    reduces the first block's bn3 backward statistics, each conv3 those of its bn2 (BNGradTap);
    every gradient must match the plain autograd path (all gradient fusions off)."""
    import hipps.models.resnet as R

    torch.manual_seed(6)
    net = torch.nn.Sequential(R.Bottleneck(64, 64, stride=1, downsample=True), R.Bottleneck(256, 64),
                              R.Bottleneck(256, 128, stride=2, downsample=True))
    net = net.to(DEV).to(memory_format=torch.channels_last)
    for blk in net:
        torch.nn.init.uniform_(blk.bn3.weight, 0.5, 1.5)
    x0 = _cl(torch.randn(8, 64, 14, 14, device=DEV).to(torch.bfloat16))
    g = None
    res = {}
    for fused in (True, False):
        R._FUSED_GRAD = fused
        R._FUSED_BNGRAD = bngrad
        try:
            net.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = net(x)
            if g is None:
                g = _cl(torch.randn(y.shape, device=DEV).to(torch.bfloat16))
            y.backward(g)
        finally:
            R._FUSED_GRAD = R._FUSED_BNGRAD = True
        res[fused] = [y.float(), x.grad.float()] + [p.grad.float().clone() for p in net.parameters()]
    for u, v in zip(res[True], res[False]):
        scale = v.abs().max().item() + 1e-6
        torch.testing.assert_close(u / scale, v / scale, rtol=0, atol=2e-2)


def test_conv1x1_bn_backward_partials_match_reduce():
    """The dgrad epilogue's BN-backward partials equal the BN reduction over the stored dy."""
    torch.manual_seed(8)
    n, c, h, w, cout = 4, 128, 10, 10, 256
    dy_out = _cl(torch.randn(n, cout, h, w, device=DEV).to(torch.bfloat16))
    wt = (torch.randn(c, cout, device=DEV) / cout ** 0.5).to(torch.bfloat16)  # [Cin, Cout] dgrad B operand
    xbn = _cl(torch.randn(n, c, h, w, device=DEV).to(torch.bfloat16))
    mean, invstd = torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5
    scale, shift = torch.randn(c, device=DEV), torch.randn(c, device=DEV)
    bits = torch.randint(0, 256, (xbn.numel() // 8,), dtype=torch.uint8, device=DEV)
    mt = native().conv1x1_mtiles(n * h * w)
    for use_bits in (True, False):
        dx = torch.empty_like(xbn)
        part = torch.empty(2, c, mt, device=DEV)
        native().conv1x1_forward(dy_out, wt, dx, part, h, w, 1, None, None, xbn, bits if use_bits else None, mean,
                                 invstd, scale, shift)
        d = dx.float().permute(0, 2, 3, 1).reshape(-1, c)
        xf = xbn.float().permute(0, 2, 3, 1).reshape(-1, c)
        if use_bits:
            m = ((bits.view(-1, 1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1).view(-1, c).bool()
        else:
            m = xf * scale + shift > 0
        dz = torch.where(m, d, torch.zeros_like(d))
        torch.testing.assert_close(part[0].sum(1), dz.sum(0), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(part[1].sum(1), (dz * (xf - mean) * invstd).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("cin,width,stride,ds", [(256, 64, 1, False), (64, 64, 1, True), (256, 128, 2, True)])
def test_bottleneck_gradient_fusions(cin, width, stride, ds):
    """Residual-gradient epilogue sums (ResidualTap for identity blocks, x alias for downsample
    blocks) only re-associate bf16 gradient sums: with a live residual branch (bn3 weight != 0)
    x.grad and every weight gradient match the autograd-add path."""
    import hipps.models.resnet as R

    torch.manual_seed(5)
    blk = R.Bottleneck(cin, width, stride=stride, downsample=ds).to(DEV).to(memory_format=torch.channels_last)
    torch.nn.init.uniform_(blk.bn3.weight, 0.5, 1.5)
    x0 = _cl(torch.randn(8, cin, 14, 14, device=DEV).to(torch.bfloat16))
    g = None
    res = {}
    for flag in (True, False):
        R._FUSED_GRAD = flag
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = blk(x)
            if g is None:
                g = _cl(torch.randn(y.shape, device=DEV).to(torch.bfloat16))
            y.backward(g)
        finally:
            R._FUSED_GRAD = True
        res[flag] = [y.float(), x.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
    for u, v in zip(res[True], res[False]):
        scale = v.abs().max().item() + 1e-6
        torch.testing.assert_close(u / scale, v / scale, rtol=0, atol=2e-2)


@pytest.mark.parametrize("cin,cout,k", [(64, 64, 3), (128, 128, 3), (256, 128, 3), (64, 32, 5)])
def test_kxk_dgrad_as_forward_matches_fp32(cin, cout, k):
    """Stride-1 'same' KxK input gradient computed as conv(dy, rot180(W)^T) (_ConvKxK) vs the
    fp32 autograd gradient of F.conv2d."""
    torch.manual_seed(cin + cout + k)
    conv = torch.nn.Conv2d(cin, cout, k, padding=k // 2, bias=False).to(DEV).to(memory_format=torch.channels_last)
    x0 = _cl(torch.randn(4, cin, 14, 14, device=DEV).to(torch.bfloat16))
    g = _cl(torch.randn(4, cout, 14, 14, device=DEV).to(torch.bfloat16))
    x = x0.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = hnn.conv2d(conv, x)
    assert y.grad_fn is not None and "ConvKxK" in type(y.grad_fn).__name__
    y.backward(g)
    xr = x0.float().requires_grad_(True)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    F.conv2d(xr, wr, padding=k // 2).backward(g.float())
    scale = xr.grad.abs().max().item()
    torch.testing.assert_close(x.grad.float() / scale, xr.grad / scale, rtol=0, atol=1e-2)
    scale = wr.grad.abs().max().item()
    torch.testing.assert_close(conv.weight.grad.float() / scale, wr.grad / scale, rtol=0, atol=1e-2)


@pytest.mark.parametrize("cin,cout,hw", [(64, 256, 14), (128, 512, 7), (256, 1024, 7)])
def test_bn_relu_prologue_matches_materialized(cin, cout, hw):
    """conv1x1 forward / weight gradient reading relu(x * scale + shift) in the operand prologue
    == the same GEMMs on the materialised bf16 BN output (the apply kernel rounds identically)."""
    from hipps.ops._native import native

    C = native()
    torch.manual_seed(cin)
    x = _cl(torch.randn(4, cin, hw, hw, device=DEV).to(torch.bfloat16))
    scale = torch.rand(cin, device=DEV) + 0.5
    shift = torch.randn(cin, device=DEV) * 0.5
    w = torch.randn(cout, cin, device=DEV).to(torch.bfloat16) * 0.05
    yref = torch.empty_like(x)
    C.bn_apply(x, None, yref, scale, shift, cin, True)
    M = 4 * hw * hw
    mt = C.conv1x1_mtiles(M)
    out_a = _cl(torch.empty(4, cout, hw, hw, device=DEV, dtype=torch.bfloat16))
    out_b = torch.empty_like(out_a)
    pa = torch.empty(2, cout, mt, device=DEV)
    pb = torch.empty_like(pa)
    C.conv1x1_forward(x, w, out_a, pa, hw, hw, 1, pro_scale=scale, pro_shift=shift)
    C.conv1x1_forward(yref, w, out_b, pb, hw, hw, 1)
    assert torch.equal(out_a, out_b) and torch.equal(pa, pb)
    dy = _cl(torch.randn(4, cout, hw, hw, device=DEV).to(torch.bfloat16))
    dwa = torch.empty(cout, cin, device=DEV)
    dwb = torch.empty_like(dwa)
    C.conv1x1_wgrad(dy, x, dwa, hw, hw, 1, scale, shift)
    C.conv1x1_wgrad(dy, yref, dwb, hw, hw, 1)
    assert torch.equal(dwa, dwb)


def test_bottleneck_bn2_prologue_matches_apply_path():
    """ResNet bottlenecks with bn2's apply in conv3's operand prologue vs the apply-kernel path:
    forward output and every gradient agree (the prologue recomputes the same bf16 values)."""
    import hipps.models.resnet as R

    torch.manual_seed(5)
    net = torch.nn.Sequential(R.Bottleneck(64, 64, stride=1, downsample=True), R.Bottleneck(256, 64),
                              R.Bottleneck(256, 128, stride=2, downsample=True))
    net = net.to(DEV).to(memory_format=torch.channels_last)
    for blk in net:
        torch.nn.init.uniform_(blk.bn3.weight, 0.5, 1.5)
    x0 = _cl(torch.randn(8, 64, 14, 14, device=DEV).to(torch.bfloat16))
    g = None
    res = {}
    for pro in (True, False):
        R._FUSED_PRO = pro
        try:
            net.zero_grad(set_to_none=True)
            for b in net.modules():
                if isinstance(b, torch.nn.BatchNorm2d):
                    b.reset_running_stats()
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = net(x)
            if g is None:
                g = _cl(torch.randn(y.shape, device=DEV).to(torch.bfloat16))
            y.backward(g)
            res[pro] = [y.detach().float(), x.grad.float()] + [p.grad.float() for p in net.parameters()]
            res[pro] += [b.running_mean.clone() for b in net.modules() if isinstance(b, torch.nn.BatchNorm2d)]
        finally:
            R._FUSED_PRO = False
    for u, v in zip(res[True], res[False]):  # MIOpen's 3x3 kernels reduce with atomics: run-to-run noise
        scale = v.abs().max().item() + 1e-6
        torch.testing.assert_close(u / scale, v / scale, rtol=0, atol=2e-2)


@pytest.mark.parametrize("c,h,stride,k", [(64, 20, 1, 3), (128, 15, 2, 3), (256, 9, 1, 3), (64, 11, 1, 5),
                                          (128, 8, 2, 1)])
def test_convkxk_forward_matches_fp32(c, h, stride, k):
    """hipps implicit-GEMM KxK forward (taps, zero padding, stride) + BN-statistics epilogue vs an
    fp32 convolution of the same bf16 operands."""
    from hipps.ops._native import native

    torch.manual_seed(c + h)
    n, cout, pad = 3, 2 * c, k // 2
    x = _cl(torch.randn(n, c, h, h, device=DEV).to(torch.bfloat16))
    w = _cl((torch.randn(cout, c, k, k, device=DEV) / (k * c ** 0.5)).to(torch.bfloat16))
    ref = torch.nn.functional.conv2d(x.float(), w.float(), stride=stride, padding=pad)
    y = _cl(torch.empty(ref.shape, device=DEV, dtype=torch.bfloat16))
    part = torch.empty(2, cout, native().conv1x1_mtiles(n * ref.shape[2] * ref.shape[3]), device=DEV)
    native().convkxk_forward(x, w, y, part, stride, pad)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    yf = y.float()
    torch.testing.assert_close(part[0].sum(1), yf.sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[1].sum(1), (yf * yf).sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
