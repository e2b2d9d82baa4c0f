"""Device-dispatching hipps ops.

Every op takes flat buffers.  HIP tensors run the hand-written gfx950 kernels in
``hipps/csrc/*.hip`` (and FAIL if the extension is not built); CPU tensors run
:mod:`hipps.ops.reference`.  Kernels are enqueued on the current HIP stream, so callers pick the
stream with ``torch.cuda.stream(...)``.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import reference as ref
from ._native import available as native_available  # noqa: F401
from ._native import native

QBLOCK = ref.QBLOCK


def _dev(t: torch.Tensor) -> bool:
    return t.is_cuda


def aggregate(slots: Sequence[torch.Tensor], acc: torch.Tensor, gscale: float = 1.0, accumulate: bool = False,
              acquire: bool = False):
    """acc (+)= gscale * sum_w slots[w], summed in rank order (reference ps.py:176).
    ``acquire``: a source was written by another GPU (async PS mailbox slot of a remote worker):
    every workgroup does a system-scope acquire before its first load (csrc/common.h)."""
    if _dev(acc):
        return native().aggregate(list(slots), acc, float(gscale), bool(accumulate), bool(acquire))
    return ref.aggregate(slots, acc, gscale, accumulate)


def copy_acquire(src: torch.Tensor, dst: torch.Tensor):
    """dst = src (uint8) after a system-scope acquire: stages bytes a peer GPU wrote into this
    device's memory before ordinary kernels read them."""
    if _dev(src):
        return native().copy_acquire(src, dst)
    dst.copy_(src)


def convert(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0):
    """dst = scale*src with f32<->bf16 conversion (wire pack / unpack)."""
    if _dev(src):
        return native().convert(src, dst, float(scale))
    return ref.convert(src, dst, scale)


def sgd_step(grads: Sequence[torch.Tensor], p: torch.Tensor, buf: Optional[torch.Tensor] = None,
             pub: Optional[torch.Tensor] = None, zero_src: bool = False, gscale: float = 1.0, lr: float = 0.0,
             weight_decay: float = 0.0, momentum: float = 0.0, dampening: float = 0.0, nesterov: bool = False,
             first: bool = False, mask: Optional[torch.Tensor] = None, csteps: Optional[torch.Tensor] = None,
             lookahead: float = 0.0):
    """Fused decode + sum_W + SGD (reference ps.py:197-214) + optional publish copy.  ``mask``
    (uint8, one byte per 16 elements) leaves chunks with a 0 byte untouched (params without a
    gradient, ps.py:178-179).  ``csteps`` (int32 per 16-element chunk) makes the first-step rule
    per parameter (buf = d_p where the chunk's count is 0) and counts the chunks it updates.
    ``lookahead`` c != 0 writes ``pub = p - c * buf`` (look-ahead publish for async readers)."""
    if _dev(p):
        return native().sgd_step(list(grads), float(gscale), p, buf, pub, bool(zero_src), float(lr),
                                 float(weight_decay), float(momentum), float(dampening), bool(nesterov), bool(first),
                                 mask, csteps, float(lookahead))
    return ref.sgd_step(list(grads), p, buf, pub, zero_src, gscale, lr, weight_decay, momentum, dampening,
                        nesterov, first, mask, csteps, lookahead)


def adam_step(grads: Sequence[torch.Tensor], p: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
              max_exp_avg_sq: Optional[torch.Tensor] = None, pub: Optional[torch.Tensor] = None,
              zero_src: bool = False, gscale: float = 1.0, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
              weight_decay: float = 0.0, step: int = 1, amsgrad: bool = False, torch_mode: bool = False,
              mask: Optional[torch.Tensor] = None, csteps: Optional[torch.Tensor] = None):
    """Fused decode + sum_W + Adam (reference ps.py:217-261 eps placement unless torch_mode).
    ``csteps`` (int32 per 16-element chunk): per-parameter step t = count + 1 for the bias
    correction (ps.py:241), advanced for the chunks it updates; ``step`` is then only the hint
    for the common t (chunks at that t use the host-computed scalars)."""
    if _dev(p):
        return native().adam_step(list(grads), float(gscale), p, exp_avg, exp_avg_sq, max_exp_avg_sq, pub,
                                  bool(zero_src), float(lr), float(betas[0]), float(betas[1]), float(eps),
                                  float(weight_decay), int(step), bool(amsgrad), bool(torch_mode), mask, csteps)
    return ref.adam_step(list(grads), p, exp_avg, exp_avg_sq, max_exp_avg_sq, pub, zero_src, gscale, lr, betas, eps,
                         weight_decay, step, amsgrad, torch_mode, mask, csteps)


def q8_encode(x, resid, q, scales, stochastic: bool = False, seed: int = 0):
    if _dev(x):
        return native().q8_encode(x, resid, q, scales, bool(stochastic), int(seed) & ((1 << 63) - 1))
    return ref.q8_encode(x, resid, q, scales, stochastic, int(seed) & ((1 << 63) - 1))


def q8_aggregate(qs, ss, acc, gscale: float = 1.0, accumulate: bool = False, acquire: bool = False):
    if _dev(acc):
        return native().q8_aggregate(list(qs), list(ss), acc, float(gscale), bool(accumulate), bool(acquire))
    return ref.q8_aggregate(qs, ss, acc, gscale, accumulate)


def topk_workspace_bytes(n: int, k: int = 0) -> int:
    """Bytes of the device workspace of a top-k (k) / threshold (k = capacity) encoder over n
    elements.  Allocate it zeroed and keep it per bucket: it carries the previous call's threshold,
    which bounds the next call's candidate list."""
    return native().topk_workspace_bytes(int(n), int(k)) if native_available() else ref.topk_workspace_bytes(n, k)


def topk_encode(g, resid, k: int, idx, val, workspace=None):
    if _dev(g):
        if workspace is None:
            workspace = torch.zeros(native().topk_workspace_bytes(g.numel(), int(k)), dtype=torch.uint8, device=g.device)
        return native().topk_encode(g, resid, int(k), idx, val, workspace)
    return ref.topk_encode(g, resid, k, idx, val)


def topk_accumulate(idx, val, acc, gscale: float = 1.0, acquire: bool = False):
    if _dev(acc):
        return native().topk_accumulate(idx, val, acc, float(gscale), bool(acquire))
    return ref.topk_accumulate(idx, val, acc, gscale)


def topk_q8_accumulate(idx, q, scales, acc, gscale: float = 1.0, acquire: bool = False):
    if _dev(acc):
        return native().topk_q8_accumulate(idx, q, scales, acc, float(gscale), bool(acquire))
    return ref.topk_q8_accumulate(idx, q, scales, acc, gscale)


def topk_q8_residual(idx, v, q, scales, resid):
    if _dev(resid):
        return native().topk_q8_residual(idx, v, q, scales, resid)
    return ref.topk_q8_residual(idx, v, q, scales, resid)


def thresh_encode(g, resid, tau: float, count, idx, val, workspace=None):
    """Variable-size sparsification: |x| > tau, capacity idx.numel(), true count in count[0]."""
    if _dev(g):
        if workspace is None:
            workspace = torch.zeros(native().topk_workspace_bytes(g.numel(), idx.numel()), dtype=torch.uint8,
                                    device=g.device)
        return native().thresh_encode(g, resid, float(tau), count, idx, val, workspace)
    return ref.thresh_encode(g, resid, tau, count, idx, val)


def thresh_accumulate(count, idx, val, acc, gscale: float = 1.0, acquire: bool = False):
    if _dev(acc):
        return native().thresh_accumulate(count, idx, val, acc, float(gscale), bool(acquire))
    return ref.thresh_accumulate(count, idx, val, acc, gscale)
