"""Fused BatchNorm(+residual)(+ReLU): CPU fallback parity and GPU kernel numerics vs fp32 torch."""
import pytest
import torch
import torch.nn.functional as F

from hipps.ops.nn import FusedBatchNorm2d


def _ref(x, res, bn, relu):
    y = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, True, bn.momentum, bn.eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


@pytest.mark.parametrize("relu,residual", [(False, False), (True, False), (True, True)])
def test_cpu_fallback_matches_batchnorm(relu, residual):
    torch.manual_seed(0)
    m = FusedBatchNorm2d(16, relu=relu)
    ref = torch.nn.BatchNorm2d(16)
    ref.load_state_dict(m.state_dict(), strict=False)
    x = torch.randn(4, 16, 5, 5)
    r = torch.randn(4, 16, 5, 5) if residual else None
    y = m(x, residual=r)
    want = ref(x) + (r if residual else 0)
    want = F.relu(want) if relu else want
    torch.testing.assert_close(y, want)
    torch.testing.assert_close(m.running_mean, ref.running_mean)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(8, 64, 56, 56), (4, 256, 14, 14), (16, 2048, 7, 7), (2, 8, 3, 3), (3, 1024, 5, 7)])
@pytest.mark.parametrize("relu,residual", [(False, False), (True, False), (True, True)])
def test_gpu_fused_bn_matches_fp32_reference(shape, relu, residual):
    torch.manual_seed(1)
    N, C, H, W = shape
    dev = "cuda"
    x0 = (torch.randn(shape, device=dev) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r0 = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last) if residual \
        else None
    m = FusedBatchNorm2d(C, relu=relu).to(dev)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    ref = FusedBatchNorm2d(C, relu=relu, fused=False).to(dev)
    ref.load_state_dict(m.state_dict())
    x = x0.clone().requires_grad_(True)
    r = r0.clone().requires_grad_(True) if residual else None
    y = m(x, residual=r)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    xf = x0.float().requires_grad_(True)
    rf = r0.float().requires_grad_(True) if residual else None
    yf = ref(xf, residual=rf)
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(m.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, ref.running_var, rtol=1e-3, atol=1e-4)
    g = torch.randn(shape, device=dev)
    y.backward(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    yf.backward(g.to(torch.bfloat16).float())
    scale = xf.grad.abs().max().item() + 1e-6
    torch.testing.assert_close(x.grad.float() / scale, xf.grad / scale, rtol=0, atol=3e-2)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, rtol=2e-2, atol=2e-2 * ref.weight.grad.abs().max().item())
    torch.testing.assert_close(m.bias.grad, ref.bias.grad, rtol=2e-2, atol=2e-2 * ref.bias.grad.abs().max().item())
    if residual:
        torch.testing.assert_close(r.grad.float(), rf.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_gpu_fused_eval_apply():
    torch.manual_seed(2)
    m = FusedBatchNorm2d(64, relu=True).cuda().eval()
    m.running_mean.uniform_(-1, 1)
    m.running_var.uniform_(0.5, 2)
    x = torch.randn(2, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(x)
        m.fused = False
        want = m(x.float())
    torch.testing.assert_close(y.float(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("width,pro", [(16, False), (64, False), (64, True), (64, 2)])
def test_gpu_resnet_fused_vs_unfused_step(width, pro, monkeypatch):
    """One autocast step of a small ResNet: the fused-BN model's grads are no further from an fp32
    reference than the eager bf16 (MIOpen BN) model's grads are.  width 64 puts every conv on the
    MFMA paths (BNGradTap through the 3x3 input gradient, the downsample's compact stride-2
    gradient summed in conv1's dgrad epilogue)."""
    import copy

    import hipps.models.resnet as rn
    from hipps.models.resnet import ResNet, Bottleneck

    monkeypatch.setattr(rn, "_BN_PRO", pro is True)  # bn1 / bn2 applied inside conv2 / conv3 (_BNReluConv)
    monkeypatch.setattr(rn, "_BN_PRO2", pro == 2)  # bn2 inside conv3 only
    torch.manual_seed(3)
    base = ResNet(Bottleneck, [1, 1], num_classes=10, width=width, zero_init_residual=False).cuda()
    base = base.to(memory_format=torch.channels_last)
    models = {k: copy.deepcopy(base) for k in ("fused", "eager", "fp32")}
    for k in ("eager", "fp32"):
        for mod in models[k].modules():
            if isinstance(mod, FusedBatchNorm2d):
                mod.fused = False
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    losses = {}
    for k, m in models.items():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(k != "fp32")):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        losses[k] = loss.item()
    assert abs(losses["fused"] - losses["fp32"]) < 3e-2
    ref = dict(models["fp32"].named_parameters())
    for k in ("fused", "eager"):
        pass
    worse = []
    for (n, pf), pe in zip(models["fused"].named_parameters(), models["eager"].parameters()):
        g = ref[n].grad
        ef = (pf.grad - g).norm().item()
        ee = (pe.grad - g).norm().item()
        if ef > 1.5 * ee + 1e-3 * g.norm().item() + 1e-6:
            worse.append((n, ef, ee))
    assert not worse, worse


@pytest.mark.gpu
def test_gpu_bn_prologue_per_layer_choice(monkeypatch):
    """bn2 -> conv3 with the BN in conv3's operand prologue (chosen per layer by a measurement,
    ops.nn.bn_pro_pays) computes the same step as the apply pass + plain GEMMs: loss, every gradient
    and the BN running statistics agree whichever way each layer goes, and the measured choice is
    cached under a 'bnpro' tuner key."""
    import copy

    import hipps.models.resnet as rn
    from hipps.models.resnet import Bottleneck, ResNet
    from hipps.ops import nn as hnn

    torch.manual_seed(4)
    cl = torch.channels_last
    base = ResNet(Bottleneck, [2, 1], num_classes=10, width=64, zero_init_residual=False).cuda().to(memory_format=cl)
    x = torch.randn(16, 3, 64, 64, device="cuda").contiguous(memory_format=cl)
    y = torch.randint(0, 10, (16,), device="cuda")
    res = {}
    for mode in ("apply", "pro", "tuned"):
        m = copy.deepcopy(base)
        if mode == "tuned":
            monkeypatch.setattr(rn, "bn_pro_pays", hnn.bn_pro_pays)
        else:
            monkeypatch.setattr(rn, "bn_pro_pays", lambda *a, _p=(mode == "pro"): _p)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        res[mode] = (loss.item(), [p.grad.clone() for p in m.parameters()],
                     [b.clone() for n, b in m.named_buffers() if "running" in n])
    assert any(k[0] == "bnpro" for k in hnn.TUNER.cache)
    for mode in ("pro", "tuned"):
        assert abs(res[mode][0] - res["apply"][0]) < 1e-3
        for a, b in zip(res[mode][1], res["apply"][1]):
            torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-3 * max(1.0, b.abs().max().item()))
        for a, b in zip(res[mode][2], res["apply"][2]):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("with_part3", [False, True])
def test_gpu_dual_bn_relu_matches_fp32(with_part3):
    """relu(bn3(x3) + bnd(xd)) on _DualBNRelu (statistics from producer partials, the downsample BN
    applied inside bn3's pass, backward in two passes) against fp32 torch BatchNorm autograd."""
    from hipps.ops import nn as hnn
    from hipps.ops._native import native

    torch.manual_seed(5)
    n, C, h = 4, 256, 9
    cl = torch.channels_last
    x3 = torch.randn(n, C, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    xd = (torch.randn(n, C, h, h, device="cuda") * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    bn3, bnd = FusedBatchNorm2d(C, relu=True).cuda(), FusedBatchNorm2d(C).cuda()
    with torch.no_grad():
        for b in (bn3, bnd):
            b.weight.uniform_(0.5, 1.5)
            b.bias.uniform_(-0.2, 0.2)

    def parts(x):  # producer-style partials [2, C, nrb] (sum, sum of squares per row block)
        xf = x.permute(0, 2, 3, 1).reshape(-1, C).float()
        blocks = xf.split(64)
        return torch.stack([torch.stack([b.sum(0) for b in blocks], 1),
                            torch.stack([(b * b).sum(0) for b in blocks], 1)]).contiguous()

    a3 = x3.clone().requires_grad_(True)
    ad = xd.clone().requires_grad_(True)
    z = hnn.dual_bn_relu(bn3, a3, parts(x3), bnd, ad, parts(xd))
    g = torch.randn_like(z)
    if with_part3:  # bn3's backward reduction delivered by the consumer (as a dgrad epilogue would)
        bg = z._hipps_bngrad
        gf = g.float().permute(0, 2, 3, 1).reshape(-1, C)
        bits = ((bg.mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).view(-1, C).bool()
        dzm = torch.where(bits, gf, torch.zeros_like(gf))
        xh = (x3.float().permute(0, 2, 3, 1).reshape(-1, C) - bg.mean) * bg.invstd
        bg.part = torch.stack([dzm.sum(0), (dzm * xh).sum(0)]).view(2, C, 1).contiguous()
    z.backward(g)
    r3, rd = torch.nn.BatchNorm2d(C).cuda(), torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        r3.weight.copy_(bn3.weight), r3.bias.copy_(bn3.bias), rd.weight.copy_(bnd.weight), rd.bias.copy_(bnd.bias)
    f3 = x3.float().requires_grad_(True)
    fd = xd.float().requires_grad_(True)
    zr = torch.relu(r3(f3) + rd(fd))
    zr.backward(g.float())
    torch.testing.assert_close(z.float(), zr, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(a3.grad.float(), f3.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(ad.grad.float(), fd.grad, rtol=3e-2, atol=3e-2)
    for mine, ref in ((bn3, r3), (bnd, rd)):
        torch.testing.assert_close(mine.weight.grad, ref.weight.grad, rtol=2e-2, atol=5e-2)
        torch.testing.assert_close(mine.bias.grad, ref.bias.grad, rtol=2e-2, atol=5e-2)
        torch.testing.assert_close(mine.running_mean, ref.running_mean, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(mine.running_var, ref.running_var, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_gpu_wgrad_side_stream_grads_ready_after_backward(monkeypatch):
    """Weight gradients computed on the side stream are complete when backward() returns: read
    straight after it on the caller's stream (as a clip_grad_norm_ would), they equal the in-line
    ones.  A second backward (accumulation into an existing .grad) takes the in-line path."""
    import copy

    import hipps.ops.nn as hnn
    from hipps.models.resnet import ResNet, Bottleneck

    torch.manual_seed(4)
    base = ResNet(Bottleneck, [1, 1], num_classes=10, width=64).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")

    def grads(side, twice=False):
        monkeypatch.setattr(hnn, "_WGRAD_SIDE", side)
        m = copy.deepcopy(base)
        for _ in range(2 if twice else 1):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                F.cross_entropy(m(x), y).backward()
        return torch.cat([p.grad.float().flatten() for p in m.parameters()])  # no synchronize first

    grads(False)  # tuner warm-up
    ref = grads(False)
    got = grads(True)
    assert hnn.wgrad_stream(0) is not None
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(grads(True, twice=True), grads(False, twice=True), rtol=1e-4, atol=1e-6)
