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
