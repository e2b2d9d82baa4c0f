"""hipps flash attention (csrc/attn.hip, hipps.ops.nn.attention) against an fp32
softmax(Q K^T / sqrt(d) + mask) V reference: forward output, log-sum-exp and all three
gradients, for the transformer configs' shapes (BERT head dim 64, Llama head dim 128 with
causal masking and grouped-query heads), odd sequence lengths and key padding.

The bf16 error is also compared with PyTorch SDPA's own bf16 error against the same fp32
reference, so the bound is not a loose absolute number."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal, kv_len, scale):
    """fp32 reference on [B, S, H, D] inputs (GQA by repetition)."""
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    rep = qf.shape[1] // kf.shape[1]
    kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    Sq, Sk = s.shape[-2], s.shape[-1]
    mask = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device)[None, None].expand(q.shape[0], 1, Sq, Sk).clone()
    if causal:
        mask &= torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril()
    if kv_len is not None:
        mask &= (torch.arange(Sk, device=q.device)[None, :] < kv_len.view(-1, 1))[:, None, None, :]
    s = s.masked_fill(~mask, float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.softmax(s, -1).nan_to_num(0.0)
    return (p @ vf).transpose(1, 2), lse


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


CASES = [
    # B, S, Hq, Hkv, D, causal, padded
    (2, 128, 4, 4, 64, False, False),
    (2, 512, 4, 4, 64, False, False),
    (1, 1000, 4, 4, 64, False, False),
    (2, 512, 4, 4, 64, False, True),
    (1, 2048, 4, 4, 64, True, False),
    (2, 128, 8, 2, 128, True, False),
    (1, 512, 8, 2, 128, True, False),
    (1, 1000, 8, 2, 128, True, False),
    (1, 2048, 8, 2, 128, True, False),
    (1, 512, 4, 4, 128, False, False),
    (1, 1000, 4, 1, 128, False, True),
    (2, 333, 8, 2, 64, True, False),
    (1, 2048, 8, 8, 128, False, False),
]


@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal,padded", CASES)
def test_flash_attention_forward_backward(B, S, Hq, Hkv, D, causal, padded):
    from hipps.ops import nn as hnn

    torch.manual_seed(S * 7 + Hq + D + int(causal))
    dev = "cuda"
    q = torch.randn(B, S, Hq, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device=dev).to(torch.bfloat16)
    kv_len = None
    if padded:
        kv_len = torch.tensor([S - 37 - 50 * i for i in range(B)], device=dev, dtype=torch.int32)
    scale = 1.0 / D ** 0.5
    assert hnn.attention_ok(q, k, v, causal)
    qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = hnn.attention(qa, ka, va, causal=causal, kv_len=kv_len)
    assert o.shape == q.shape and o.dtype == torch.bfloat16
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref, lse_ref = _ref(qr, kr, vr, causal, kv_len, scale)
    # forward
    assert _rel(o, ref) < 1.5e-2, _rel(o, ref)
    _, lse = hnn.native().attn_forward(q, k, v, causal, scale, kv_len)
    ok = torch.isfinite(lse_ref)
    torch.testing.assert_close(lse[ok], lse_ref[ok], rtol=1e-3, atol=2e-3)
    # backward
    g = torch.randn_like(o)
    o.backward(g)
    ref.backward(g.float())
    for got, want, name in ((qa.grad, qr.grad, "dq"), (ka.grad, kr.grad, "dk"), (va.grad, vr.grad, "dv")):
        assert got.shape == want.shape and got.dtype == torch.bfloat16, name
        assert torch.isfinite(got.float()).all(), name
        assert _rel(got, want) < 3e-2, (name, _rel(got, want))
    if padded:  # masked keys get no gradient
        for i in range(B):
            assert torch.count_nonzero(ka.grad[i, int(kv_len[i]):]) == 0
            assert torch.count_nonzero(va.grad[i, int(kv_len[i]):]) == 0


@pytest.mark.parametrize("causal,Hkv,D", [(False, 4, 64), (True, 2, 128)])
def test_flash_attention_error_vs_sdpa(causal, Hkv, D):
    """hipps' bf16 error against fp32 is no worse than 1.5x PyTorch SDPA's bf16 error."""
    from hipps.ops import nn as hnn
    import torch.nn.functional as F

    torch.manual_seed(11)
    B, S, Hq = 2, 512, 8
    q = torch.randn(B, S, Hq, D, device="cuda").to(torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda").to(torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda").to(torch.bfloat16)
    ref, _ = _ref(q, k, v, causal, None, D ** -0.5)
    rep = Hq // Hkv
    sd = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2).repeat_interleave(rep, 1),
                                        v.transpose(1, 2).repeat_interleave(rep, 1), is_causal=causal).transpose(1, 2)
    ours = hnn.attention(q, k, v, causal=causal)
    assert _rel(ours, ref) <= 1.5 * _rel(sd, ref) + 1e-3, (_rel(ours, ref), _rel(sd, ref))


def test_flash_attention_deterministic_and_strided_inputs():
    """Backward is bitwise repeatable (no atomics), and q / k / v may be strided views of a fused
    [B, S, 3, H, D] projection."""
    from hipps.ops import nn as hnn

    torch.manual_seed(5)
    B, S, H, D = 2, 384, 6, 64
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    assert not q.is_contiguous() and hnn.attention_ok(q, k, v)
    g = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
    grads = []
    for _ in range(2):
        x = qkv.clone().requires_grad_(True)
        o = hnn.attention(x[:, :, 0], x[:, :, 1], x[:, :, 2])
        o.backward(g)
        grads.append((o.detach(), x.grad))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    ref, _ = _ref(q, k, v, False, None, D ** -0.5)
    assert _rel(grads[0][0], ref) < 1.5e-2


def test_flash_attention_in_models(monkeypatch):
    """BERT and Llama blocks (head dims 64 / 128, Llama causal + GQA) route attention to the hipps
    kernels and match their SDPA route's loss and gradients."""
    from hipps.ops import nn as hnn
    from hipps.models import transformer as tf

    calls = []
    for cls in (hnn._FlashAttention, hnn._FlashAttentionQKV, hnn._RopeAttentionPacked):  # BERT / Llama packed
        def counted(ctx, *a, _fwd=cls.forward):
            calls.append(1)
            return _fwd(ctx, *a)

        monkeypatch.setattr(cls, "forward", staticmethod(counted))
    torch.manual_seed(0)
    models = [(tf.Bert(tf.BertConfig(vocab=512, hidden=128, layers=2, heads=2, ffn=256, max_pos=128)), 2),
              (tf.Llama(tf.LlamaConfig(vocab=512, dim=256, layers=2, heads=2, kv_heads=1, ffn=256, max_seq=128)), 2)]
    for m, nlayers in models:
        m = m.cuda()
        ids = torch.randint(0, 512, (2, 96), device="cuda")
        outs = []
        for fused in (True, False):
            monkeypatch.setattr(hnn, "_FUSED_ATTN", fused)
            calls.clear()
            m.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(ids, labels=ids)
            loss.backward()
            assert len(calls) == (nlayers if fused else 0)
            outs.append((loss.detach().float(), [p.grad.detach().float().clone() for p in m.parameters()
                                                  if p.grad is not None]))
        (l1, g1), (l0, g0) = outs
        torch.testing.assert_close(l1, l0, rtol=2e-2, atol=2e-2)
        num = sum((a - b).norm() ** 2 for a, b in zip(g1, g0)) ** 0.5
        den = sum(b.norm() ** 2 for b in g0) ** 0.5
        assert num / den < 5e-2, num / den


@pytest.mark.parametrize("padded", [False, True])
def test_packed_qkv_attention_matches_separate(padded):
    """attention_qkv (one packed [B, S, 3, H, D] input, its gradient written packed by the kernels)
    equals attention on the three views, forward and backward, bit for bit."""
    from hipps.ops import nn as hnn

    torch.manual_seed(21)
    B, S, H, D = 2, 320, 4, 64
    base = torch.randn(B, S, 3 * H * D, device="cuda").to(torch.bfloat16)
    kv_len = torch.tensor([S, S - 77], device="cuda", dtype=torch.int32) if padded else None
    g = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
    x1 = base.clone().requires_grad_(True)
    o1 = hnn.attention_qkv(x1.view(B, S, 3, H, D), kv_len=kv_len)
    o1.backward(g)
    x2 = base.clone().requires_grad_(True)
    q, k, v = x2.view(B, S, 3, H, D).unbind(2)
    o2 = hnn.attention(q, k, v, kv_len=kv_len)
    o2.backward(g)
    assert torch.equal(o1, o2)
    assert torch.equal(x1.grad, x2.grad)


@pytest.mark.parametrize("D,hq,hkv", [(64, 8, 2), (128, 4, 1)])
def test_rope_attention_packed_matches_separate_path(D, hq, hkv):
    """Llama's packed q | k | v projection: RoPE + causal GQA attention with the gradient written
    packed and rotated back in place equals rope() + attention() on the three slices, bit for bit."""
    from hipps.ops import nn as hnn
    from hipps.models.transformer import _rope

    torch.manual_seed(D + hq)
    B, S = 2, 256
    W = (hq + 2 * hkv) * D
    base = (torch.randn(B, S, W, device="cuda") * 0.5).to(torch.bfloat16)
    inv = 1.0 / (5e5 ** (torch.arange(0, D, 2, device="cuda", dtype=torch.float32) / D))
    f = torch.outer(torch.arange(S, device="cuda", dtype=torch.float32), inv)
    cos, sin = f.cos().contiguous(), f.sin().contiguous()
    g = torch.randn(B, S, hq, D, device="cuda").to(torch.bfloat16)
    y1 = base.clone().requires_grad_(True)
    assert hnn.rope_attention_packed_ok(y1, cos, hq, hkv)
    o1 = hnn.rope_attention_packed(y1, cos, sin, hq, hkv)
    o1.backward(g)
    y2 = base.clone().requires_grad_(True)
    q, k, v = y2.split([hq * D, hkv * D, hkv * D], dim=-1)
    q, k = q.reshape(B, S, hq, D).contiguous(), k.reshape(B, S, hkv, D).contiguous()
    assert hnn.rope_ok(q, cos) and hnn.rope_ok(k, cos)  # (the same RoPE kernel on both paths)
    q, k = _rope(q, cos, sin), _rope(k, cos, sin)
    o2 = hnn.attention(q, k, v.reshape(B, S, hkv, D), causal=True)
    o2.backward(g)
    assert torch.equal(o1, o2)
    assert torch.equal(y1.grad, y2.grad)


def test_swiglu_packed_matches_fp32_and_unpacked():
    from hipps.ops import nn as hnn
    import torch.nn.functional as F

    torch.manual_seed(2)
    y = (torch.randn(3, 77, 2 * 384, device="cuda") * 2).to(torch.bfloat16)
    g = torch.randn(3, 77, 384, device="cuda").to(torch.bfloat16)
    yp = y.clone().requires_grad_(True)
    c = hnn.swiglu_packed(yp)
    c.backward(g)
    a, b = y.float().split(384, dim=-1)
    a.requires_grad_(True)
    b.requires_grad_(True)
    ref = F.silu(a) * b
    ref.backward(g.float())
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(yp.grad.float(), torch.cat([a.grad, b.grad], -1), rtol=2e-2, atol=2e-2)
    a2, b2 = (t.contiguous().requires_grad_(True) for t in y.split(384, dim=-1))
    c2 = hnn.swiglu(a2, b2)
    c2.backward(g)
    assert torch.equal(c, c2) and torch.equal(yp.grad, torch.cat([a2.grad, b2.grad], -1))
