"""CPU tests of the reference op semantics (the oracle the GPU kernels are checked against).

SGD/Adam are checked against independent re-statements of the reference formulas
(/root/reference/ps.py:197-214, 217-261) written out step by step here.
"""
import math

import numpy as np
import pytest
import torch

from hipps import ops
from hipps.ops import reference as ref


def _ref_sgd_loop(p, grads_seq, lr, wd, mom, damp, nesterov):
    """Literal transcription of ps.py SGD.optim_step (per-parameter state dict)."""
    state = {}
    p = p.clone()
    for d_p in grads_seq:
        d_p = d_p.clone()
        if wd != 0:
            d_p.add_(p, alpha=wd)
        if mom != 0:
            if "momentum_buffer" not in state:
                buf = state["momentum_buffer"] = torch.zeros_like(p)
                buf.mul_(mom).add_(d_p)
            else:
                buf = state["momentum_buffer"]
                buf.mul_(mom).add_(d_p, alpha=1 - damp)
            if nesterov:
                d_p = d_p.add(buf, alpha=mom)
            else:
                d_p = buf
        p.add_(d_p, alpha=-lr)
    return p


@pytest.mark.parametrize("mom,damp,nesterov,wd", [(0, 0, False, 0), (0.9, 0, False, 1e-4), (0.9, 0.1, False, 0),
                                                  (0.9, 0, True, 5e-4)])
def test_sgd_reference_matches_ps_py(mom, damp, nesterov, wd):
    torch.manual_seed(0)
    n = 1000
    p0 = torch.randn(n)
    seq = [torch.randn(n) for _ in range(4)]
    want = _ref_sgd_loop(p0, seq, 0.1, wd, mom, damp, nesterov)
    p = p0.clone()
    buf = torch.zeros(n)
    for t, g in enumerate(seq):
        ops.sgd_step([g], p, buf if mom else None, lr=0.1, weight_decay=wd, momentum=mom, dampening=damp,
                     nesterov=nesterov, first=(t == 0))
    torch.testing.assert_close(p, want, rtol=0, atol=0)


def _ref_adam_loop(p, seq, lr, betas, eps, wd, amsgrad):
    """Literal transcription of ps.py Adam.optim_step."""
    p = p.clone()
    st = {"step": 0, "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p),
          "max_exp_avg_sq": torch.zeros_like(p)}
    for grad in seq:
        b1, b2 = betas
        st["step"] += 1
        if wd != 0:
            grad = grad.add(p, alpha=wd)
        st["exp_avg"].mul_(b1).add_(grad, alpha=1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(grad, grad, value=1 - b2)
        if amsgrad:
            torch.max(st["max_exp_avg_sq"], st["exp_avg_sq"], out=st["max_exp_avg_sq"])
            denom = st["max_exp_avg_sq"].sqrt().add_(eps)
        else:
            denom = st["exp_avg_sq"].sqrt().add_(eps)
        bc1 = 1 - b1 ** st["step"]
        bc2 = 1 - b2 ** st["step"]
        step_size = lr * math.sqrt(bc2) / bc1
        p.addcdiv_(st["exp_avg"], denom, value=-step_size)
    return p


@pytest.mark.parametrize("amsgrad,wd", [(False, 0.0), (True, 1e-2)])
def test_adam_reference_matches_ps_py(amsgrad, wd):
    torch.manual_seed(1)
    n = 777
    p0 = torch.randn(n)
    seq = [torch.randn(n) for _ in range(5)]
    want = _ref_adam_loop(p0, seq, 1e-2, (0.9, 0.999), 1e-8, wd, amsgrad)
    p, m, v, vm = p0.clone(), torch.zeros(n), torch.zeros(n), torch.zeros(n)
    for t, g in enumerate(seq, 1):
        ops.adam_step([g], p, m, v, vm if amsgrad else None, lr=1e-2, betas=(0.9, 0.999), eps=1e-8,
                      weight_decay=wd, step=t, amsgrad=amsgrad)
    torch.testing.assert_close(p, want, rtol=0, atol=0)


def test_adam_torch_mode_matches_torch_optim():
    torch.manual_seed(2)
    n = 300
    p0 = torch.randn(n)
    seq = [torch.randn(n) for _ in range(3)]
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([tp], lr=1e-2)
    for g in seq:
        tp.grad = g.clone()
        opt.step()
    p, m, v = p0.clone(), torch.zeros(n), torch.zeros(n)
    for t, g in enumerate(seq, 1):
        ops.adam_step([g], p, m, v, lr=1e-2, step=t, torch_mode=True)
    torch.testing.assert_close(p, tp.detach(), rtol=1e-6, atol=1e-7)


def test_aggregate_rank_order_and_bf16():
    torch.manual_seed(3)
    slots = [torch.randn(100).to(torch.bfloat16) for _ in range(3)]
    acc = torch.zeros(100)
    ops.aggregate(slots, acc, 0.5)
    want = (slots[0].float() + slots[1].float() + slots[2].float()) * 0.5
    torch.testing.assert_close(acc, want)
    ops.aggregate(slots[:1], acc, 1.0, accumulate=True)
    torch.testing.assert_close(acc, want + slots[0].float())


def test_q8_roundtrip_and_error_feedback():
    torch.manual_seed(4)
    n = 1000  # not a multiple of the 256 block
    x = torch.randn(n)
    q = torch.empty(n, dtype=torch.int8)
    s = torch.empty((n + 255) // 256)
    r = torch.zeros(n)
    ops.q8_encode(x, r, q, s)
    deq = ref.q8_dequant(q, s)
    # error feedback invariant: x == deq + r exactly in the math (fp32 rounding only)
    torch.testing.assert_close(deq + r, x, rtol=0, atol=1e-6)
    assert (deq - x).abs().max() <= s.max() / 2 + 1e-6
    assert q.abs().max() <= 127


def test_q8_stochastic_rounding_unbiased():
    x = torch.full((256 * 64,), 0.3)
    x[0] = 1.0  # pins the block scale
    q = torch.empty_like(x, dtype=torch.int8)
    s = torch.empty(64)
    ops.q8_encode(x, None, q, s, stochastic=True, seed=123)
    deq = ref.q8_dequant(q, s)
    assert abs(deq[1:256].mean().item() - 0.3) < 0.02


def test_topk_reference_ties_and_order():
    x = torch.tensor([0.5, -3.0, 2.0, -2.0, 2.0, 0.1, 3.0])
    sel = ref.topk_select(x, 4)
    # |x|: 3.0 at 1 and 6, 2.0 at 2,3,4 -> lowest-index tie break takes 2,3
    assert sel.tolist() == [1, 2, 3, 6]
    idx = torch.empty(4, dtype=torch.int32)
    val = torch.empty(4)
    r = torch.zeros(7)
    ops.topk_encode(x, r, 4, idx, val)
    assert idx.tolist() == [1, 2, 3, 6]
    assert val.tolist() == [-3.0, 2.0, -2.0, 3.0]
    # EF residual keeps exactly the untransmitted mass
    torch.testing.assert_close(r, torch.tensor([0.5, 0, 0, 0, 2.0, 0.1, 0]))
    acc = torch.zeros(7)
    ops.topk_accumulate(idx, val, acc)
    torch.testing.assert_close(acc + r, x)


def test_uniform01_matches_splitmix_definition():
    u = ref.uniform01(7, np.arange(4, dtype=np.int64))
    assert u.dtype == np.float32 and ((u >= 0) & (u < 1)).all()
    assert len(set(u.tolist())) == 4


def test_threshold_codec_variable_size_and_ef():
    from hipps.codecs import Threshold

    x = torch.tensor([0.5, -3.0, 0.01, 2.0, -0.2, 0.0, 1.0])
    c = Threshold(tau=0.3, max_ratio=0.5)  # capacity 4
    lay = c.layout(7)
    buf = torch.zeros(lay.nbytes, dtype=torch.uint8)
    v = lay.views(buf)
    st = c.init_state(7, "cpu")
    c.encode_into(x, v, st)
    assert int(v["count"][0]) == 4 and v["idx"].tolist() == [0, 1, 3, 6]
    acc = torch.zeros(7)
    c.accumulate([v], acc)
    torch.testing.assert_close(acc + st["resid"], x)
    # capacity clamps: a second, denser message keeps the overflow in the residual
    c2 = Threshold(tau=0.0, max_ratio=2 / 7, error_feedback=False)
    lay2 = c2.layout(7)
    v2 = lay2.views(torch.zeros(lay2.nbytes, dtype=torch.uint8))
    c2.encode_into(x, v2, c2.init_state(7, "cpu"))
    assert int(v2["count"][0]) == 2 and v2["idx"].tolist() == [0, 1]
