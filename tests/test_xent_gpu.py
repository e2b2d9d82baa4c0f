"""Fused softmax cross-entropy of bf16 logits (csrc/xent.hip, hipps.ops.nn.cross_entropy) against
PyTorch's fp32 route, F.cross_entropy(logits.float()), incl. ignored rows and vocab sizes that are
not a multiple of 8 (unaligned rows, scalar tail)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,vocab", [(64, 1000), (37, 30522), (8, 128256), (5, 13), (3, 7)])
def test_fused_cross_entropy_matches_fp32(rows, vocab):
    from hipps.ops import nn as hnn

    torch.manual_seed(rows + vocab)
    x = (torch.randn(rows, vocab, device="cuda") * 3).to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, vocab, (rows,), device="cuda")
    if rows > 4:
        y[1] = -100
        y[rows - 2] = -100
    x0 = x.detach().float().requires_grad_(True)
    loss = hnn.cross_entropy(x, y)
    loss0 = F.cross_entropy(x0, y, ignore_index=-100)
    torch.testing.assert_close(loss.float(), loss0, rtol=1e-4, atol=1e-4)
    loss.backward(torch.tensor(2.0, device="cuda"))
    loss0.backward(torch.tensor(2.0, device="cuda"))
    assert x.grad.dtype == torch.bfloat16
    torch.testing.assert_close(x.grad.float(), x0.grad, rtol=1e-2, atol=2e-3 / max(1, rows // 8))
    if rows > 4:
        assert torch.count_nonzero(x.grad[1]) == 0


def test_fused_cross_entropy_in_3d_lm_head_layout():
    """[batch, seq, vocab] logits from a head GEMM, mean over every token."""
    from hipps.ops import nn as hnn

    torch.manual_seed(9)
    x = torch.randn(2, 16, 515, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, 515, (2, 16), device="cuda")
    loss = hnn.cross_entropy(x, y)
    loss0 = F.cross_entropy(x.detach().float().view(-1, 515), y.view(-1))
    torch.testing.assert_close(loss.float(), loss0, rtol=1e-4, atol=1e-4)
    loss.backward()
    assert x.grad.shape == x.shape and torch.isfinite(x.grad.float()).all()


@pytest.mark.parametrize("rows,cols", [(16384, 768), (333, 3072), (5, 8), (1, 64), (4097, 1000)])
def test_colsum_matches_fp32(rows, cols):
    from hipps.ops import nn as hnn

    torch.manual_seed(rows)
    t = torch.randn(rows, cols, device="cuda").to(torch.bfloat16)
    got = hnn.colsum_f32(t)
    ref = t.double().sum(0)
    assert got.dtype == torch.float32
    torch.testing.assert_close(got.double(), ref, rtol=1e-5, atol=1e-3)
    assert torch.equal(got, hnn.colsum_f32(t))  # deterministic


def test_colsum_one_launch_tickets_rearm():
    """The column sum (two launches by default; with HIPPS_COLSUM_ONE=1 the one-launch form whose
    last-arriving block per column tile folds, xent.hip): many calls of different shapes on two
    streams, each right and bitwise repeatable (the one-launch form's counters re-arm)."""
    from hipps.ops import nn as hnn

    torch.manual_seed(1)
    ts = [torch.randn(r, c, device="cuda").to(torch.bfloat16) for r, c in
          ((16384, 768), (16384, 3072), (100, 64), (4097, 2304), (1, 8))]
    refs = [t.double().sum(0) for t in ts]
    first = [hnn.colsum_f32(t) for t in ts]
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    for i in range(40):
        k = i % len(ts)
        with torch.cuda.stream(side if i % 3 == 0 else torch.cuda.current_stream()):
            got = hnn.colsum_f32(ts[k])
        torch.cuda.synchronize()
        torch.testing.assert_close(got.double(), refs[k], rtol=1e-5, atol=1e-3)
        assert torch.equal(got, first[k])


def test_fused_cross_entropy_label_semantics():
    """the mean counts only rows that carry a loss.  Ignored rows and out-of-range
    labels (which F.cross_entropy rejects) are excluded from the denominator; every row ignored
    gives NaN, as F.cross_entropy does."""
    from hipps.ops.nn import cross_entropy

    torch.manual_seed(3)
    logits = torch.randn(8, 64, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 64, (8,), device="cuda")
    y[1] = -100
    y[5] = -100
    ref = torch.nn.functional.cross_entropy(logits.float(), y, ignore_index=-100)
    got = cross_entropy(logits, y)
    torch.testing.assert_close(got.float(), ref, rtol=1e-3, atol=1e-3)
    bad = y.clone()
    bad[2] = 64  # out of range: no loss, not counted
    keep = (bad != -100) & (bad < 64)
    ref2 = torch.nn.functional.cross_entropy(logits.float()[keep], bad[keep])
    torch.testing.assert_close(cross_entropy(logits, bad).float(), ref2, rtol=1e-3, atol=1e-3)
    allign = torch.full_like(y, -100)
    assert torch.isnan(cross_entropy(logits, allign)) and torch.isnan(
        torch.nn.functional.cross_entropy(logits.float(), allign))


@pytest.mark.parametrize("vocab", [30522, 30521, 30515])
def test_fused_cross_entropy_unaligned_rows_every_row(vocab):
    """Rows of an odd-sized vocab start at every 2-byte offset from a 16-byte boundary; the
    kernels peel each row's head to the boundary and keep the vector loop.  Every row's loss and
    gradient against F.cross_entropy(logits.float(), reduction='none')."""
    from hipps.ops import nn as hnn

    torch.manual_seed(vocab)
    rows = 67
    x = (torch.randn(rows, vocab, device="cuda") * 4).to(torch.bfloat16)
    y = torch.randint(0, vocab, (rows,), device="cuda")
    y[0], y[1], y[2] = 0, vocab - 1, 3  # labels in the peeled head and in the scalar tail
    xr = x.clone().requires_grad_(True)
    x0 = x.float().requires_grad_(True)
    loss = hnn.cross_entropy(xr, y)
    per_row = F.cross_entropy(x0, y, reduction="none")
    torch.testing.assert_close(loss.float(), per_row.mean(), rtol=1e-4, atol=1e-4)
    per_row.mean().backward()
    loss.backward()
    g, g0 = xr.grad.float(), x0.grad
    err = ((g - g0).abs() / (g0.abs() + 2e-3 / rows)).amax(dim=1)
    assert (err < 2e-2).all(), err.max()
    # per-row log-sum-exp saved by the forward vs fp32 logsumexp, every row
    _, _, lse = hnn.native().xent_forward(x, y, -100)
    torch.testing.assert_close(lse, torch.logsumexp(x.float(), dim=1), rtol=1e-5, atol=1e-4)
