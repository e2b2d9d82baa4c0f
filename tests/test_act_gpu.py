"""Fused Llama-block elementwise kernels (csrc/act.hip) against plain PyTorch fp32 references:
the SwiGLU gate silu(a) * b and the rotary embedding, forward and backward."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("shape", [(8, 64), (4096, 8192), (3, 5, 136)])
def test_swiglu_matches_fp32(shape):
    from hipps.ops import nn as hnn

    torch.manual_seed(sum(shape))
    a = (torch.randn(shape, device=DEV) * 3).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(shape, device=DEV).to(torch.bfloat16).requires_grad_(True)
    c = hnn.swiglu(a, b)
    assert c.grad_fn is not None and "SwiGLU" in type(c.grad_fn).__name__
    af, bf = a.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    ref = F.silu(af) * bf
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2)
    g = torch.randn(shape, device=DEV).to(torch.bfloat16)
    c.backward(g)
    ref.backward(g.float())
    torch.testing.assert_close(a.grad.float(), af.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(b.grad.float(), bf.grad, rtol=2e-2, atol=2e-2)


def _rope_ref(x, cos, sin):
    S = x.shape[1]
    c, s = cos[None, :S, None, :], sin[None, :S, None, :]
    x1, x2 = x[..., ::2], x[..., 1::2]
    return torch.stack((x1 * c - x2 * s, x1 * s + x2 * c), dim=-1).flatten(-2)


@pytest.mark.parametrize("B,S,H,hd", [(2, 16, 4, 16), (4, 2048, 8, 128), (1, 33, 3, 64)])
def test_rope_matches_fp32(B, S, H, hd):
    from hipps.ops import nn as hnn

    torch.manual_seed(S + H)
    inv = 1.0 / (5e5 ** (torch.arange(0, hd, 2, device=DEV, dtype=torch.float32) / hd))
    f = torch.outer(torch.arange(S, device=DEV, dtype=torch.float32), inv)
    cos, sin = f.cos().contiguous(), f.sin().contiguous()
    x = torch.randn(B, S, H, hd, device=DEV).to(torch.bfloat16).requires_grad_(True)
    assert hnn.rope_ok(x, cos)
    y = hnn.rope(x, cos, sin)
    xf = x.detach().float().requires_grad_(True)
    ref = _rope_ref(xf, cos, sin)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=1e-2, atol=1e-2)


def test_llama_tiny_fused_act_matches_eager():
    """A llama-tiny forward + backward under autocast with the fused SwiGLU / RoPE vs the eager ops."""
    from hipps.models.transformer import build
    from hipps.ops import nn as hnn

    def run(fused):
        saved = hnn._FUSED_ACT
        hnn._FUSED_ACT = fused
        try:
            torch.manual_seed(7)
            m = build("llama-tiny").to(DEV)
            ids = torch.randint(0, 512, (2, 64), device=DEV, generator=torch.Generator(device=DEV).manual_seed(8))
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(ids, ids)
            loss.backward()
            return loss.item(), torch.cat([p.grad.flatten() for p in m.parameters()])
        finally:
            hnn._FUSED_ACT = saved

    (l1, g1), (l0, g0) = run(True), run(False)
    assert abs(l1 - l0) < 2e-2
    torch.testing.assert_close(g1, g0, rtol=5e-2, atol=5e-3)


@pytest.mark.parametrize("R,D", [(16384, 768), (33, 64), (100, 2048), (7, 520)])
def test_layer_norm_matches_fp32(R, D):
    """csrc/ln.hip LayerNorm (bf16 rows, fp32 affine params) against F.layer_norm in fp32: output,
    input gradient and the fp32 weight / bias gradients; the backward is deterministic."""
    from hipps.ops import nn as hnn

    torch.manual_seed(R + D)
    x = (torch.randn(R, D, device=DEV) * 2 + 0.5).to(torch.bfloat16).requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.2 + 1)
    b = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.1)
    assert hnn.layer_norm_ok(x, w, b)
    y = hnn.layer_norm(x, w, b, 1e-12)
    xf = x.detach().float().requires_grad_(True)
    wf, bf = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    ref = F.layer_norm(xf, (D,), wf, bf, 1e-12)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn(R, D, device=DEV).to(torch.bfloat16)
    y.backward(g)
    ref.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=3e-2, atol=3e-2)
    assert w.grad.dtype == torch.float32 and b.grad.dtype == torch.float32
    tol = 2e-3 * R ** 0.5 + 1e-3
    torch.testing.assert_close(w.grad, wf.grad, rtol=2e-2, atol=tol)
    torch.testing.assert_close(b.grad, bf.grad, rtol=2e-2, atol=tol)
    w.grad = b.grad = x.grad = None
    hnn.layer_norm(x, w, b, 1e-12).backward(g)
    dw1 = w.grad.clone()
    w.grad = None
    hnn.layer_norm(x, w, b, 1e-12).backward(g)
    assert torch.equal(dw1, w.grad)


def test_bert_tiny_fused_norm_matches_eager():
    """bert-tiny forward + backward under autocast with the hipps LayerNorm vs F.layer_norm."""
    from hipps.models.transformer import build
    from hipps.ops import nn as hnn

    def run(fused):
        saved = hnn._FUSED_ACT
        hnn._FUSED_ACT = fused
        try:
            torch.manual_seed(9)
            m = build("bert-tiny").to(DEV)
            ids = torch.randint(0, 512, (4, 32), device=DEV, generator=torch.Generator(device=DEV).manual_seed(10))
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(ids, ids)
            loss.backward()
            return loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])
        finally:
            hnn._FUSED_ACT = saved

    (l1, g1), (l0, g0) = run(True), run(False)
    assert abs(l1 - l0) < 2e-2
    torch.testing.assert_close(g1, g0, rtol=5e-2, atol=5e-3)


@pytest.mark.parametrize("R,D,dtype", [(8192, 2048, torch.float32), (2048, 4096, torch.float32), (33, 64, torch.bfloat16),
                                       (100, 4096, torch.bfloat16), (7, 1000 // 8 * 8, torch.float32)])
def test_rms_norm_matches_fp32(R, D, dtype):
    """csrc/ln.hip RMSNorm (fp32 or bf16 rows -> bf16, fp32 weight) against the fp32 formula: output,
    input gradient in x's dtype and the fp32 weight gradient; deterministic backward."""
    from hipps.ops import nn as hnn

    torch.manual_seed(R + D)
    x = (torch.randn(R, D, device=DEV) * 3).to(dtype).requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.2 + 1)
    assert hnn.rms_norm_ok(x, w)
    y = hnn.rms_norm(x, w, 1e-5)
    assert y.dtype == torch.bfloat16
    xf = x.detach().float().requires_grad_(True)
    wf = w.detach().clone().requires_grad_(True)
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn(R, D, device=DEV).to(torch.bfloat16)
    y.backward(g)
    ref.backward(g.float())
    assert x.grad.dtype == dtype and w.grad.dtype == torch.float32
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad, wf.grad, rtol=2e-2, atol=2e-3 * R ** 0.5 + 1e-3)
    w.grad = None
    hnn.rms_norm(x, w, 1e-5).backward(g)
    dw1 = w.grad.clone()
    w.grad = None
    hnn.rms_norm(x, w, 1e-5).backward(g)
    assert torch.equal(dw1, w.grad)


@pytest.mark.parametrize("R,D,with_dres", [(8192, 2048, True), (2048, 4096, True), (33, 64, False), (7, 1000 // 8 * 8, True)])
def test_add_rms_norm_matches_fp32(R, D, with_dres):
    """csrc/ln.hip fused residual add + RMSNorm: s = x + y (fp32 x, bf16 y), bf16 norm(s); the
    backward returns the fp32 residual gradient (incoming ds + norm backward, one pass) for x and
    its bf16 twin for y, against the fp32 formula."""
    from hipps.ops import nn as hnn

    torch.manual_seed(R + D + 1)
    x = (torch.randn(R, D, device=DEV) * 3).requires_grad_(True)
    y = torch.randn(R, D, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(D, device=DEV) * 0.2 + 1)
    assert hnn.add_rms_norm_ok(x, y, w)
    s, h = hnn.add_rms_norm(x, y, w, 1e-5)
    assert s.dtype == torch.float32 and h.dtype == torch.bfloat16
    xf, yf = x.detach().clone().requires_grad_(True), y.detach().float().requires_grad_(True)
    wf = w.detach().clone().requires_grad_(True)
    sf = xf + yf
    ref = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    torch.testing.assert_close(s, sf, rtol=0, atol=0)
    torch.testing.assert_close(h.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn(R, D, device=DEV).to(torch.bfloat16)
    gs = torch.randn(R, D, device=DEV) if with_dres else None
    if with_dres:
        torch.autograd.backward((s, h), (gs, g))
        torch.autograd.backward((sf, ref), (gs, g.float()))
    else:
        h.backward(g)
        ref.backward(g.float())
    assert x.grad.dtype == torch.float32 and y.grad.dtype == torch.bfloat16
    torch.testing.assert_close(x.grad, xf.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.grad.float(), xf.grad.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    assert torch.equal(y.grad, x.grad.to(torch.bfloat16))
    torch.testing.assert_close(w.grad, wf.grad, rtol=2e-2, atol=2e-3 * R ** 0.5 + 1e-3)


def test_layer_norm_dx_colsum_stash():
    """LayerNorm backward with colsum_dx: the column sum of the bf16 dx it wrote is left for
    colsum_f32 (the bias gradient of the Linear before the norm) -- equal to summing dx itself,
    consumed once, and voided by an in-place change of dx.  (dx is caught by a hook on a non-leaf
    input, as the Linear's backward receives it: a leaf's .grad may be a copy.)"""
    from hipps.ops import nn as hnn

    torch.manual_seed(4)
    R, D = 4096, 768
    x0 = torch.randn(R, D, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = torch.randn(D, device=DEV) * 0.2 + 1
    b = torch.randn(D, device=DEV) * 0.1
    g = torch.randn(R, D, device=DEV).to(torch.bfloat16)

    def run():
        got = []
        x = x0 * 1.0
        x.register_hook(lambda t: got.append(t))
        hnn.layer_norm(x, w, b, 1e-12, colsum_dx=True).backward(g)
        return got[0]

    dx = run()
    assert dx.data_ptr() in hnn._COLSUM_STASH
    ref = dx.double().sum(0)
    got = hnn.colsum_f32(dx)
    torch.testing.assert_close(got.double(), ref, rtol=1e-5, atol=1e-3)
    assert dx.data_ptr() not in hnn._COLSUM_STASH  # consumed
    dx = run()
    dx.mul_(2)  # in-place change: the stashed sum is void
    torch.testing.assert_close(hnn.colsum_f32(dx).double(), dx.double().sum(0), rtol=1e-5, atol=1e-3)
