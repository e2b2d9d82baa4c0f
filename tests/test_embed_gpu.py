"""csrc/embed.hip: BERT's word + position + token-type embedding (hnn.bert_embed) against the fp64
formula -- forward (bf16 rounding of the fp32 sum, PyTorch's add order) and every table gradient
(duplicate ids summed, unused ids zero, position rows past S zero); deterministic backward; the
BERT model with the fused embedding against its PyTorch-embedding route."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("B,S,V,P,D,typed", [(4, 100, 50, 128, 64, False), (8, 512, 30522, 512, 768, False),
                                             (3, 33, 7, 40, 136, True), (2, 64, 1, 64, 8, True)])
def test_bert_embed_matches_fp64(B, S, V, P, D, typed):
    from hipps.ops import nn as hnn

    torch.manual_seed(B * S + V)
    word = torch.nn.Parameter(torch.randn(V, D, device=DEV))
    pos = torch.nn.Parameter(torch.randn(P, D, device=DEV))
    typ = torch.nn.Parameter(torch.randn(2, D, device=DEV))
    ids = torch.randint(0, V, (B, S), device=DEV)
    tt = torch.randint(0, 2, (B, S), device=DEV) if typed else None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert hnn.bert_embed_ok(ids, word, pos, typ)
        y = hnn.bert_embed(ids, word, pos, typ, tt)
    assert y.dtype == torch.bfloat16 and y.shape == (B, S, D)
    t0 = torch.zeros_like(ids) if tt is None else tt
    ref32 = (word[ids] + pos[:S][None]) + typ[t0]
    assert torch.equal(y, ref32.detach().to(torch.bfloat16))
    g = torch.randn(B, S, D, device=DEV).to(torch.bfloat16)
    y.backward(g)
    wd, pd, td = (p.detach().double().requires_grad_(True) for p in (word, pos, typ))
    ((wd[ids] + pd[:S][None]) + td[t0]).backward(g.double())
    for p, r in ((word, wd), (pos, pd), (typ, td)):
        assert p.grad.dtype == torch.float32
        torch.testing.assert_close(p.grad.double(), r.grad, rtol=1e-5, atol=1e-4)
    grads = [p.grad.clone() for p in (word, pos, typ)]
    for p in (word, pos, typ):
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        hnn.bert_embed(ids, word, pos, typ, tt).backward(g)
    assert all(torch.equal(a, p.grad) for a, p in zip(grads, (word, pos, typ)))


def test_bert_tiny_fused_embedding_matches_pytorch_route(monkeypatch):
    from hipps.models.transformer import build
    from hipps.ops import nn as hnn

    def run(fused):
        monkeypatch.setattr(hnn, "_FUSED_EMBED", fused)
        torch.manual_seed(11)
        m = build("bert-tiny").to(DEV)
        ids = torch.randint(0, 512, (4, 32), device=DEV, generator=torch.Generator(device=DEV).manual_seed(12))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(ids, ids)
        loss.backward()
        return loss.item(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    (l1, g1), (l0, g0) = run(True), run(False)
    assert abs(l1 - l0) < 1e-3
    assert g1.keys() == g0.keys()
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n], rtol=2e-2, atol=2e-3, msg=n)
