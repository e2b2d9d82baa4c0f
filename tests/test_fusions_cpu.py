"""CPU checks of the round-6 fusion plumbing (the device kernels have GPU tests; these pin the
Python-side contracts every path relies on): the column-sum stash (consumed once, voided by an
in-place change, bounded), the residual link and the GELU MLP falling back to the module
compositions, RMSNorm's deferred residual add, and the Llama block's deferred residual structure
against a direct implementation of the same math."""
import torch
import torch.nn.functional as F

from hipps.ops import nn as hnn


def test_colsum_stash_contract():
    hnn._COLSUM_STASH.clear()
    t = torch.randn(64, 16)
    cs = torch.full((16,), 7.0)
    hnn.stash_colsum(t, cs)
    assert hnn.colsum_f32(t) is cs  # the producer's sum, no pass over t
    torch.testing.assert_close(hnn.colsum_f32(t), t.sum(0))  # consumed: computed again
    hnn.stash_colsum(t, cs)
    t.mul_(2)  # in-place change voids it
    torch.testing.assert_close(hnn.colsum_f32(t), t.sum(0))
    ts = [torch.randn(8, 8) for _ in range(6)]
    for x in ts:
        hnn.stash_colsum(x, torch.zeros(8))
    assert len(hnn._COLSUM_STASH) == 4  # bounded: the oldest entries dropped
    assert ts[0].data_ptr() not in hnn._COLSUM_STASH and ts[-1].data_ptr() in hnn._COLSUM_STASH
    hnn._COLSUM_STASH.clear()


def test_residual_link_and_gelu_mlp_fall_back_on_cpu():
    torch.manual_seed(0)
    l1, l2, l3 = hnn.Linear(16, 32), hnn.Linear(32, 16), hnn.Linear(16, 16)
    x = torch.randn(4, 5, 16, requires_grad=True)
    x0 = x.detach().clone().requires_grad_(True)
    link = hnn.ResidualLink()
    y = l3(torch.tanh(l1(x, link=link)[..., :16]), residual=x, link=link) + hnn.gelu_mlp(x, l1, l2, residual_x=True)
    y0 = (l3(torch.tanh(l1(x0)[..., :16])) + x0) + (l2(F.gelu(l1(x0))) + x0)
    torch.testing.assert_close(y, y0)
    g = torch.randn_like(y)
    y.backward(g)
    y0.backward(g)
    torch.testing.assert_close(x.grad, x0.grad)
    assert link.g is None and not link.armed  # never armed off the shadow path


def test_rmsnorm_deferred_residual_add():
    from hipps.models.transformer import RMSNorm

    torch.manual_seed(1)
    n = RMSNorm(32, 1e-5)
    with torch.no_grad():
        n.weight.uniform_(0.5, 1.5)
    x, y = torch.randn(3, 7, 32), torch.randn(3, 7, 32)
    s, h = n(x, add=y)
    torch.testing.assert_close(s, x + y)
    torch.testing.assert_close(h, n(x + y))


def test_llama_deferred_residuals_match_direct_blocks():
    """Llama.forward carries (x, pending branch output) between blocks and folds each add into the
    next norm; the result must equal the plain pre-norm residual formulation."""
    from hipps.models.transformer import build

    torch.manual_seed(2)
    m = build("llama-tiny")
    ids = torch.randint(0, 512, (2, 16))
    got = m(ids)
    B, S = ids.shape
    c = m.c
    hd = c.dim // c.heads
    cos, sin = m.rope_tables(S, ids.device)
    x = m.tok(ids)
    for b in m.blocks:
        h = b.attn_norm(x)
        q, k, v = b.wqkv(h).split([c.heads * hd, c.kv_heads * hd, c.kv_heads * hd], dim=-1)
        from hipps.models.transformer import _rope

        q = _rope(q.reshape(B, S, c.heads, hd), cos, sin)
        k = _rope(k.reshape(B, S, c.kv_heads, hd), cos, sin)
        a = hnn.attention(q, k, v.reshape(B, S, c.kv_heads, hd), causal=True)
        x = x + b.wo(a.reshape(B, S, c.dim))
        h = b.ffn_norm(x)
        g13 = b.w13(h)
        x = x + b.w2(F.silu(g13[..., :c.ffn]) * g13[..., c.ffn:])
    ref = m.head(m.norm(x))
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_bert_embed_gate_is_device_only():
    w = torch.randn(10, 8)
    ids = torch.randint(0, 10, (2, 4))
    assert not hnn.bert_embed_ok(ids, w, torch.randn(4, 8), torch.randn(2, 8))
