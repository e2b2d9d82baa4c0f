"""Pure-PyTorch reference implementations of every hipps kernel.

Two roles:
  * the CPU backend (gloo plumbing tests, BASELINE config 1 "MLP sync PS on CPU");
  * the numerics oracle the GPU kernel tests compare against (fp32 torch math).

Semantics mirror the HIP kernels exactly (rank-ordered sums, reference SGD/Adam formulas from
/root/reference/ps.py:197-261, 256-element int8 blocks, exact top-k with lowest-index tie
break, ascending index order).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch

QBLOCK = 256


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.float()


def aggregate(slots: Sequence[torch.Tensor], acc: torch.Tensor, gscale: float = 1.0, accumulate: bool = False):
    if accumulate:  # each message added on its own (batch-invariant; csrc/flat.hip k_aggregate)
        for s in slots:
            acc.add_(_f32(s) * gscale if gscale != 1.0 else _f32(s))
        return
    d = _f32(slots[0]).clone()
    for s in slots[1:]:  # rank order (ps.py:176 `sum(grads)`)
        d += _f32(s)
    if gscale != 1.0:
        d *= gscale
    if accumulate:
        acc += d
    else:
        acc.copy_(d)


def convert(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0):
    x = _f32(src)
    if scale != 1.0:
        x = x * scale
    dst.copy_(x.to(dst.dtype))


def _elem_mask(mask, n):
    """Chunk mask (one byte per 16 elements) -> per-element bool."""
    return mask.bool().repeat_interleave(16)[:n]


def _masked(mask, n, fn, *bufs):
    """Run ``fn`` and restore the elements of ``bufs`` whose chunk mask byte is 0."""
    if mask is None:
        return fn()
    keep = ~_elem_mask(mask, n)
    saved = [b[keep].clone() if b is not None else None for b in bufs]
    fn()
    for b, s in zip(bufs, saved):
        if b is not None:
            b[keep] = s


def _chunk_groups(mask, csteps, key):
    """Split the chunks this step updates (mask byte != 0, or all) by ``key(count)`` -> list of
    (key value, chunk mask) so each group runs the scalar-hyper-parameter formula."""
    live = torch.ones_like(csteps, dtype=torch.bool) if mask is None else mask[: csteps.numel()].to(torch.bool)
    keys = key(csteps)
    out = []
    for kv in sorted(set(keys[live].tolist())):
        out.append((kv, (live & (keys == kv)).to(torch.uint8)))
    return live, out


def sgd_step(grads, p, buf=None, pub=None, zero_src=False, gscale=1.0, lr=0.0, weight_decay=0.0, momentum=0.0,
             dampening=0.0, nesterov=False, first=False, mask=None, csteps=None, lookahead=0.0):
    """Reference SGD (ps.py:197-214) on flat fp32 buffers; masked chunks are left untouched.
    ``csteps``: per-chunk update counts -- first step (buf = d_p) where the count is 0.
    ``lookahead`` c: the published copy is ``p - c * buf``."""
    if lookahead:
        sgd_step(grads, p, buf, None, zero_src, gscale, lr, weight_decay, momentum, dampening, nesterov, first, mask,
                 csteps)
        if pub is not None:
            pub.copy_(p.add(buf, alpha=-lookahead).to(pub.dtype))
        return
    if csteps is not None:
        live, groups = _chunk_groups(mask, csteps, lambda c: (c == 0).to(torch.int32))
        for is_first, m in groups:
            sgd_step(grads, p, buf, None, False, gscale, lr, weight_decay, momentum, dampening, nesterov,
                     bool(is_first), m)
        csteps[live] += 1
        if zero_src:
            grads[0].zero_()
        if pub is not None:
            pub.copy_(p.to(pub.dtype))
        return
    if mask is not None:
        _masked(mask, p.numel(), lambda: sgd_step(grads, p, buf, None, zero_src, gscale, lr, weight_decay, momentum,
                                                  dampening, nesterov, first), p, buf)
        if pub is not None:
            pub.copy_(p.to(pub.dtype))
        return
    d = _f32(grads[0]).clone()
    for g in grads[1:]:
        d += _f32(g)
    if gscale != 1.0:
        d *= gscale
    if zero_src:
        grads[0].zero_()
    if weight_decay != 0:
        d = d.add(p, alpha=weight_decay)
    if momentum != 0:
        if first:
            buf.copy_(d)
        else:
            buf.mul_(momentum).add_(d, alpha=1 - dampening)
        d = d.add(buf, alpha=momentum) if nesterov else buf
    p.add_(d, alpha=-lr)
    if pub is not None:
        pub.copy_(p.to(pub.dtype))


def adam_step(grads, p, exp_avg, exp_avg_sq, max_exp_avg_sq=None, pub=None, zero_src=False, gscale=1.0, lr=1e-3,
              betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, step=1, amsgrad=False, torch_mode=False, mask=None,
              csteps=None):
    """Reference Adam (ps.py:217-261): denom = sqrt(v) + eps; step = lr*sqrt(bc2)/bc1.
    ``csteps``: per-chunk update counts -- each chunk is corrected for its own t = count + 1."""
    if csteps is not None:
        live, groups = _chunk_groups(mask, csteps, lambda c: c + 1)
        for t, m in groups:
            adam_step(grads, p, exp_avg, exp_avg_sq, max_exp_avg_sq, None, False, gscale, lr, betas, eps,
                      weight_decay, int(t), amsgrad, torch_mode, m)
        csteps[live] += 1
        if zero_src:
            grads[0].zero_()
        if pub is not None:
            pub.copy_(p.to(pub.dtype))
        return
    if mask is not None:
        _masked(mask, p.numel(), lambda: adam_step(grads, p, exp_avg, exp_avg_sq, max_exp_avg_sq, None, zero_src,
                                                   gscale, lr, betas, eps, weight_decay, step, amsgrad, torch_mode),
                p, exp_avg, exp_avg_sq, max_exp_avg_sq)
        if pub is not None:
            pub.copy_(p.to(pub.dtype))
        return
    g = _f32(grads[0]).clone()
    for x in grads[1:]:
        g += _f32(x)
    if gscale != 1.0:
        g *= gscale
    if zero_src:
        grads[0].zero_()
    b1, b2 = betas
    if weight_decay != 0:
        g = g.add(p, alpha=weight_decay)
    exp_avg.mul_(b1).add_(g, alpha=1 - b1)
    exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
    v = exp_avg_sq
    if amsgrad:
        torch.maximum(max_exp_avg_sq, exp_avg_sq, out=max_exp_avg_sq)
        v = max_exp_avg_sq
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    if torch_mode:
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        step_size = lr / bc1
    else:
        denom = v.sqrt().add_(eps)
        step_size = lr * math.sqrt(bc2) / bc1
    p.addcdiv_(exp_avg, denom, value=-step_size)
    if pub is not None:
        pub.copy_(p.to(pub.dtype))


# ---- counter-based RNG identical to common.h uniform01 ------------------------------------
_M64 = (1 << 64) - 1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def uniform01(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = _splitmix64(np.uint64(seed & _M64) ^ (idx.astype(np.uint64) * np.uint64(0xD1B54A32D192ED03)))
    return (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def q8_encode(x, resid, q, scales, stochastic=False, seed=0):
    v = _f32(x).clone()
    if resid is not None:
        v += resid
    n = v.numel()
    nb = (n + QBLOCK - 1) // QBLOCK
    pad = nb * QBLOCK - n
    vb = torch.cat([v, v.new_zeros(pad)]).view(nb, QBLOCK)
    amax = vb.abs().amax(dim=1)
    scale = amax / 127.0
    inv = torch.where(amax > 0, 127.0 / amax, torch.zeros_like(amax))
    y = vb * inv[:, None]
    if stochastic:
        u = torch.from_numpy(uniform01(seed, np.arange(nb * QBLOCK, dtype=np.int64))).view(nb, QBLOCK)
        y = torch.floor(y + u)
    else:
        y = torch.round(y)  # rintf: round-half-even, same as torch.round
    y = y.clamp_(-127, 127).to(torch.int8)
    q.copy_(y.view(-1)[:n])
    scales.copy_(scale)
    if resid is not None:
        resid.copy_(v - y.view(-1)[:n].float() * scale.repeat_interleave(QBLOCK)[:n])


def q8_dequant(q, scales):
    n = q.numel()
    return q.float() * scales.float().repeat_interleave(QBLOCK)[:n]


def q8_aggregate(qs, ss, acc, gscale=1.0, accumulate=False):
    if accumulate:  # each message added on its own (batch-invariant; csrc/quant.hip k_q8_aggregate)
        for q, s in zip(qs, ss):
            acc.add_(q8_dequant(q, s) * gscale)
        return
    d = q8_dequant(qs[0], ss[0])
    for q, s in zip(qs[1:], ss[1:]):
        d += q8_dequant(q, s)
    if gscale != 1.0:
        d *= gscale
    if accumulate:
        acc += d
    else:
        acc.copy_(d)


def topk_select(x: torch.Tensor, k: int):
    """Exact top-k by |x| with lowest-index tie break; returns ascending indices."""
    key = x.float().abs()
    # sort by (-|x|, index): stable sort on -key keeps lowest index first among equals
    order = torch.sort(-key, stable=True).indices[:k]
    return torch.sort(order).values


def topk_encode(g, resid, k, idx, val, workspace=None):
    x = _f32(g).clone()
    if resid is not None:
        x += resid
    sel = topk_select(x, k)
    idx.copy_(sel.to(torch.int32))
    v = x[sel]
    val.copy_(v.to(val.dtype))
    if resid is not None:
        resid.copy_(x)
        resid[sel] = v - val.float()


def topk_accumulate(idx, val, acc, gscale=1.0):
    acc.index_add_(0, idx.long(), val.float() * gscale)


def topk_q8_accumulate(idx, q, scales, acc, gscale=1.0):
    acc.index_add_(0, idx.long(), q8_dequant(q, scales) * gscale)


def topk_q8_residual(idx, v, q, scales, resid):
    resid.index_add_(0, idx.long(), v.float() - q8_dequant(q, scales))


def topk_workspace_bytes(n: int, k: int = 0) -> int:
    return 16


def thresh_encode(g, resid, tau, count, idx, val, workspace=None):
    """Every |x| > tau in ascending index order, at most idx.numel() of them (count in count[0])."""
    x = _f32(g).clone()
    if resid is not None:
        x += resid
    cap = idx.numel()
    sel = torch.nonzero(x.abs() > abs(tau)).view(-1)[:cap]
    count[0] = sel.numel()
    idx[: sel.numel()] = sel.to(torch.int32)
    v = x[sel]
    val[: sel.numel()] = v.to(val.dtype)
    if resid is not None:
        resid.copy_(x)
        resid[sel] = v - val[: sel.numel()].float()


def thresh_accumulate(count, idx, val, acc, gscale=1.0):
    k = min(int(count[0]), idx.numel())
    acc.index_add_(0, idx[:k].long(), val[:k].float() * gscale)
