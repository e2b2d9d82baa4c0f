"""Fused model ops backed by hipps HIP kernels.

``conv_bn`` runs a 1x1 convolution feeding such a BN as an MFMA GEMM whose epilogue emits the
BN batch statistics (hipps/csrc/gemm.hip).

``FusedBatchNorm2d`` is a drop-in ``nn.BatchNorm2d`` that can also apply a residual add and a
ReLU in the same pass (``forward(x, residual=None)``).  On a HIP device with a channels-last
bf16 input (the autocast ResNet path) it runs hipps/csrc/norm.hip: one statistics pass, one
apply pass, and a backward that recomputes the ReLU mask instead of storing it.  Anything
else (CPU, fp32, NCHW, odd channel counts, eval with grad) takes the standard PyTorch path, so
models stay portable and the CPU test suite exercises the same module.
"""
from __future__ import annotations

import collections
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._native import native

import os as _os

# weight gradient of the MFMA 1x1 path: own split-M kernel (1, default; v2 beats MIOpen on the
# ResNet-50 shapes, profiles/conv1x1_wgrad_v2.json) or MIOpen (0), for A/B runs
_OWN_WGRAD = _os.environ.get("HIPPS_CONV_WGRAD", "1") != "0"
# stride-1 "same" KxK input gradient as a forward convolution of dy with the flipped, transposed
# weight: MIOpen's backward-data solvers zero-fill dx first (SubTensorOpWithScalar1d, ~0.47 ms per
# ResNet-50 step) and run slower than its forward kernels on the same shapes
_DGRAD_AS_FWD = _os.environ.get("HIPPS_DGRAD_FWD", "1") != "0"
# KxK forward (and the stride-1 input gradient run as a forward conv) on hipps' implicit-GEMM MFMA
# kernel, with the following BN's statistics in its epilogue, instead of MIOpen/CK.  Opt-in: it
# beats MIOpen's immediate-mode choice on every ResNet-50 3x3 shape, but not the kernels MIOpen's
# Find picks under cudnn.benchmark (bench A/B: 25.26 vs 24.90 ms of kernels per step,
# profiles/ab_r2/own_kxk_*)
_OWN_KXK_FWD = _os.environ.get("HIPPS_OWN_KXK", "0") != "0"
# ResNet stem (7x7/s2/p3, 3 -> 64 channels): forward + BN statistics and weight gradient on the
# hipps MFMA stem kernels (stem.hip) instead of MIOpen
_OWN_STEM = _os.environ.get("HIPPS_OWN_STEM", "1") != "0"

# second-generation GEMM core (gemm2.hip: LDS-DMA staging, 128x64 .. 256x256 tiles) for the 1x1
# convolutions and the KxK forward / stride-1 input gradient; per shape the fastest of {gemm2
# tiles, first core / MIOpen} is picked on first use (timed on the real operands) and cached
_GEMM2 = _os.environ.get("HIPPS_GEMM2", "1") != "0"
# downsample blocks: the stride-2 1x1 input gradient as a compact GEMM summed on conv1's even rows
# (S2Tap) instead of MIOpen's zero-filled full-size gradient
_S2TAP = _GEMM2 and _os.environ.get("HIPPS_S2TAP", "1") != "0"
# stride-2 3x3 input gradient as four output-parity GEMMs (gemm2_dgrad_s2), measured against MIOpen.
# Opt-in: the tuner picks it on two of the three layers by < 2 %, but the step is 0.07 ms slower
# with it (same-box A/B 11099 on vs 11131 img/s off, profiles/r3b/ab/)
_DGRAD_S2 = _GEMM2 and _os.environ.get("HIPPS_DGRAD_S2", "0") != "0"

MASK_NONE, MASK_X, MASK_Y, MASK_BITS = 0, 1, 2, 3

# weight gradients on a side stream: a conv's dw only feeds its gradient bucket, so it runs beside
# the input-gradient / BatchNorm-backward chain (which the rest of the backward waits on) instead of
# in series with it (ResNet-50 bs256: 23.0 -> 22.0 ms/step, profiles/r3b/ab_wgs).  The bucket encode
# waits for the side stream (engine.encode_bucket), and the caller's stream joins it at the end of
# every backward (an autograd final callback), so whatever reads .grad after backward() -- step(),
# clipping -- sees finished gradients.  Only for a parameter whose .grad is None, without tensor
# hooks, and whose dw has the parameter's layout: autograd then stores dw as is (no accumulate or
# layout copy on the main stream that would read it early).
_WGRAD_SIDE = _os.environ.get("HIPPS_WGRAD_STREAM", "1") != "0"
_WG_PRIO = int(_os.environ.get("HIPPS_WGRAD_PRIO", "0"))  # (A/B: -1 = the high-priority stream pool)
# MIOpen's backward-weights solvers may accumulate with atomics (not bitwise reproducible run to
# run); the hipps weight-gradient kernels sum their split-M slabs in a fixed order.  MIOpen is a
# tuner candidate for the 64-channel KxK weight gradients only with HIPPS_MIOPEN_WGRAD=1 (it won
# no ResNet-50 bs256 shape in round 5, profiles/r5/gemm/tuner_r5n.txt; it did win a tiny test
# shape and made two bit-identical runs differ)
_MIOPEN_WGRAD = _os.environ.get("HIPPS_MIOPEN_WGRAD", "0") != "0"
# nn.Linear on the bf16 weight shadow with an fp32 weight gradient (_ShadowLinear); 0: F.linear
_SHADOW_LINEAR = _os.environ.get("HIPPS_SHADOW_LINEAR", "1") != "0"
# softmax cross-entropy of bf16 logits on csrc/xent.hip (hipps.ops.nn.cross_entropy); 0: PyTorch
_FUSED_XENT = _os.environ.get("HIPPS_FUSED_XENT", "1") != "0"
# residual adds of the transformer output projections inside the Linear (A/B: 0 = a separate add)
_LINEAR_RESIDUAL = _os.environ.get("HIPPS_LINEAR_RESIDUAL", "1") != "0"
# SwiGLU gate and rotary embedding of the Llama block as one HIP pass each (csrc/act.hip)
_FUSED_ACT = _os.environ.get("HIPPS_FUSED_ACT", "1") != "0"
# the fused GELU MLP node (_GeluMLP: GELU in the GEMM epilogues) and the residual-gradient links
# (ResidualLink); HIPPS_GELU_MLP=0 / HIPPS_RES_LINK=0 restore the module compositions for A/B runs
_GELU_MLP = _os.environ.get("HIPPS_GELU_MLP", "1") != "0"
_RES_LINK = _os.environ.get("HIPPS_RES_LINK", "1") != "0"
# ResNet bn2 -> conv3: the BN apply + ReLU in conv3's operand prologue per layer, where measured
# faster than the apply pass + plain GEMMs (bn_pro_pays); 0: always the apply pass
_BN_PRO_TUNE = _os.environ.get("HIPPS_BN_PRO_TUNE", "1") != "0"
# _StemBlock backward (HIPPS_FUSED_STEMBWD=2, the default): the BN input gradient written by one
# elementwise pass on the recomputed pool gradient, read by the plain stem weight gradient (=1:
# recomputed inside the weight gradient's staging instead; 0: no _StemBlock, the pool gradient and
# the BN backward materialised)
_STEM_BWD_DY = _os.environ.get("HIPPS_FUSED_STEMBWD", "2") == "2"
# ... its pool-gradient recompute over 2x2 pixel blocks (one window gather per four pixels); 0: per pixel
_STEM_QUAD = _os.environ.get("HIPPS_STEM_QUAD", "1") != "0"
_WG_STREAMS: dict = {}
_WG_JOINED: dict = {}  # device -> autograd graph task whose end joins the side stream


def wgrad_stream(device):
    """The weight-gradient side stream of ``device`` if one was used, else None."""
    idx = device.index if isinstance(device, torch.device) else device
    return _WG_STREAMS.get(idx)


def _same_layout(a, b):
    return a.shape == b.shape and all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


def _joined(idx):
    """The caller's stream now waits for the side stream: every input held for the side stream's
    kernels may go back to the allocator (any later reuse of their blocks -- by allocations on the
    caller's stream, the stream they belong to -- is ordered after those kernels)."""
    _WG_UNJOINED.discard(idx)
    h = _WG_HOLD.get(idx)
    if h:
        h.clear()


def _join_wgrad(idx):
    torch.cuda.current_stream(idx).wait_stream(_WG_STREAMS[idx])
    _joined(idx)


def join_wgrad_stream(device):
    """Make the current stream of ``device`` wait for its weight-gradient side stream."""
    idx = device.index if isinstance(device, torch.device) else device
    side = _WG_STREAMS.get(idx)
    if side is not None:
        torch.cuda.current_stream(idx).wait_stream(side)
        _joined(idx)


_WG_UNJOINED: set = set()  # devices whose side stream took work after the last backward's join
# devices whose gradient consumer orders itself after the side stream (the async PS engine's
# bucket encode waits for it per bucket): no end-of-backward join into the caller's stream, so
# the next step's pull and forward run beside the last weight gradients (stem, layer 1)
_WG_DEFER: set = set()


def set_wgrad_join_deferred(device, on: bool) -> None:
    idx = device.index if isinstance(device, torch.device) else device
    if on:
        _WG_DEFER.add(idx)
    else:
        _WG_DEFER.discard(idx)


def wgrad_join_deferred(device) -> bool:
    idx = device.index if isinstance(device, torch.device) else device
    return idx in _WG_DEFER


def set_deterministic(on: bool = True) -> None:
    """Bit-for-bit repeatable training steps.  hipps' own kernels already reduce in a fixed order
    once the tuner has picked (its picks -- e.g. a weight gradient's slab count -- are made once per
    process and shape), and the MIOpen weight-gradient candidate stays out of the tuner unless
    HIPPS_MIOPEN_WGRAD=1; what remains are the MIOpen convolutions the tuner still measures against
    the hipps kernels (forward / input gradient of some KxK layers, the strided input gradients),
    whose default algorithms are not run-to-run deterministic (two runs of a ResNet differed in
    every parameter, tools/diag/determinism_probe.py).  This restricts them to MIOpen's
    deterministic algorithms (torch.backends.cudnn.deterministic); no measurable cost on the
    ResNet-50 bs256 headline (profiles/r5/det).

    Scope: a step is repeatable for a given set of tuner picks.  The picks are timed per process,
    and some candidates are not bitwise equal to each other (weight-gradient slab counts, the BN
    operand-prologue route ``bnpro``), so two processes can choose differently on a near tie.  For
    bit-for-bit runs across processes or ranks, record the picks once (``TUNER.save(path)``) and
    load them everywhere (``TUNER.load(path)`` or ``HIPPS_TUNER_CACHE=path``)."""
    torch.backends.cudnn.deterministic = bool(on)
# Inputs of in-flight side-stream weight gradients, with an event after each: kept referenced until
# the event has passed or the caller's stream joined the side stream, then dropped.  This replaces
# record_stream(): the caching allocator held every such activation-sized block back until a
# side-stream event it records at free time had passed, and, with the side stream trailing the
# main stream, kept creating new segments for the blocks still pending (~2.4 per step, 250 MB/step
# of reserved memory growth with no end, profiles/r4/r4j/alloc_probe_*.txt)
_WG_HOLD: dict = {}
_WG_SEEN: dict = {}  # device -> (graph task id, ids of the parameters whose dw went to the side stream)


def wgrad_join_pending(device) -> bool:
    """True if the weight-gradient side stream of ``device`` may hold work that no backward's final
    callback has joined into the caller's stream yet."""
    idx = device.index if isinstance(device, torch.device) else device
    return idx in _WG_UNJOINED


def _on_wgrad_stream(param, tensors, fn):
    """fn() (allocates and returns dw) on the weight-gradient side stream when enabled and
    ``param`` takes dw as is; ``tensors`` (its inputs) are recorded on that stream."""
    if not (_WGRAD_SIDE and param is not None and param.grad is None and tensors[0].is_cuda
            and not param._backward_hooks):
        if param is not None and param.grad is not None and tensors[0].is_cuda:
            # autograd will add this dw to the existing .grad on the caller's stream: with the
            # end-of-backward join deferred, that .grad may still be in flight on the side stream
            idx = tensors[0].device.index
            if idx in _WG_DEFER and idx in _WG_UNJOINED:
                torch.cuda.current_stream(tensors[0].device).wait_stream(_WG_STREAMS[idx])
                _joined(idx)
        return fn()
    dev = tensors[0].device
    idx = dev.index
    side = _WG_STREAMS.get(idx)
    if side is None:
        side = _WG_STREAMS[idx] = torch.cuda.Stream(device=dev, priority=_WG_PRIO)
    cur = torch.cuda.current_stream(dev)
    # a weight used twice in one graph (weight sharing): autograd sums its gradient contributions
    # on the caller's stream before the single AccumulateGrad, so from the second one on the
    # caller's stream waits for the side stream (covering the earlier contributions too)
    task = torch._C._current_graph_task_id()
    seen = _WG_SEEN.get(idx)
    if seen is None or seen[0] != task:
        seen = _WG_SEEN[idx] = (task, set())
    repeat = id(param) in seen[1]
    seen[1].add(id(param))
    side.wait_stream(cur)
    _WG_UNJOINED.add(idx)
    with torch.cuda.stream(side):
        out = fn()
    hold = _WG_HOLD.get(idx)
    if hold is None:
        hold = _WG_HOLD[idx] = collections.deque()
    while hold and hold[0][0].query():  # earlier weight gradients that have finished
        hold.popleft()
    ev = torch.cuda.Event()
    ev.record(side)
    hold.append((ev, tensors))
    if repeat or out.dtype != param.dtype or not _same_layout(out, param):
        cur.wait_stream(side)  # autograd sums / copies dw on this stream
        _joined(idx)
    else:
        if task < 0:  # not inside an autograd backward pass
            cur.wait_stream(side)
            _joined(idx)
        elif _WG_JOINED.get(idx) != task and idx not in _WG_DEFER:
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _join_wgrad(idx))
            _WG_JOINED[idx] = task
    return out


_TUNE_QUIET: list = []  # context-manager factories that keep other GPU work off while timing


def add_tune_quiet(fn) -> None:
    """Register ``fn() -> context manager`` to be entered around every tuner measurement (the
    co-located async PS registers a pause of its thread: its kernels would otherwise share the GPU
    with the timed candidates and skew the picks)."""
    _TUNE_QUIET.append(fn)


def remove_tune_quiet(fn) -> None:
    if fn in _TUNE_QUIET:
        _TUNE_QUIET.remove(fn)


class _Tuner:
    """Per-shape kernel choice by measurement (like cudnn.benchmark): on the first call for a
    key, every candidate runs once to warm up; then, with the device drained and the registered
    background work held (add_tune_quiet), ROUNDS rounds each time every candidate (2 calls between
    HIP events, candidates interleaved) and the fastest by its best round is cached.  Interleaved
    rounds and the minimum keep a transient neighbour (another stream's kernels) from deciding a
    pick: with the co-located PS running free a measured 35 % slower set of weight-gradient
    tilings was once picked (profiles/r5/emu/).  Candidates must be side-effect free apart from
    writing their output (every candidate writes the same values)."""

    ROUNDS = 3

    def __init__(self):
        self.cache: dict = {}
        self.times: dict = {}

    def pick(self, key, cands: dict) -> str:
        got = self.cache.get(key)
        if got is not None:
            return got
        if len(cands) == 1:
            got = next(iter(cands))
        else:
            import contextlib

            for fn in cands.values():
                fn()
            with contextlib.ExitStack() as quiet:
                for q in list(_TUNE_QUIET):
                    try:
                        quiet.enter_context(q())
                    except Exception:  # (a quiet hook that cannot hold: measure anyway)
                        pass
                # drain every stream first: kernels still running on another stream (the weight-
                # gradient side stream, the PS stream) would otherwise share the GPU with the timing
                torch.cuda.synchronize()
                evs = {name: [] for name in cands}
                for _ in range(self.ROUNDS):
                    for name, fn in cands.items():
                        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        s.record()
                        fn()
                        fn()
                        e.record()
                        evs[name].append((s, e))
                torch.cuda.synchronize()
            t = {name: min(s.elapsed_time(e) for s, e in pairs) / 2 for name, pairs in evs.items()}
            got = min(t, key=t.get)
            self.times[key] = t
        self.cache[key] = got
        return got

    def save(self, path: str) -> None:
        """Write every pick (key -> candidate name) as JSON."""
        import json

        with open(path, "w") as f:
            json.dump([[list(k), v] for k, v in self.cache.items()], f)

    def load(self, path: str) -> int:
        """Adopt recorded picks (they win over measuring): runs that load the same file make the
        same choices, so choices between candidates that are not bitwise equal (weight-gradient
        slab counts, the BN prologue route) cannot differ between runs or ranks.  Returns the
        number of picks loaded."""
        import json

        with open(path) as f:
            for k, v in json.load(f):
                self.cache[tuple(k)] = v
        return len(self.cache)


TUNER = _Tuner()
# HIPPS_TUNER_CACHE=<file>: picks recorded by TUNER.save are loaded at import (set_deterministic)
if _os.environ.get("HIPPS_TUNER_CACHE") and _os.path.exists(_os.environ["HIPPS_TUNER_CACHE"]):
    TUNER.load(_os.environ["HIPPS_TUNER_CACHE"])
# (block rows, block cols, LDS stages): 3 stages keep one tile's DMA in flight across every
# K-loop barrier (gemm2.hip k_gemm NS).  Only 128x64 keeps two blocks per CU with 3 stages; the
# others drop to one wave per SIMD and lose (profiles/gemm2_probe_r3_stages.json).  (256, 256, 5):
# the ping-pong schedule of the 256x256 tile (gemm2.hip k_gemm NS == 5)
_G2_TILES = ((128, 128, 2), (256, 256, 2), (256, 256, 5), (128, 64, 2), (256, 64, 2), (128, 64, 3))


def _g2_names(N: int):
    return [f"g2_{bm}x{bn}" + ("" if ns == 2 else f"s{ns}") for bm, bn, ns in _G2_TILES if N % bn == 0]


def _g2_parse(name: str):
    """'g2_256x128s3' -> (256, 128, 3); 'g2_128x64' -> (128, 64, 2)"""
    t = name[3:]
    ns = 2
    if "s" in t:
        t, ns = t.split("s")
    bm, bn = (int(v) for v in t.split("x"))
    return bm, bn, int(ns)


def _conv1x1_gemm(x2, w2d, y, Hi, Wi, stride, part_needed, add=None, add_mask=None, bg=None, add_s2=False):
    """y = x . w2d^T as a 1x1 conv (x channels-last [n, K, Hi, Wi] or [M, K]; w2d [N, K]) on the
    fastest core for this shape AND epilogue (candidates are timed with the real epilogue: the
    memory-bound residual / BN-backward epilogues change the ranking); returns the statistics
    partials [2, N, mtiles] if requested (the forward BN statistics, or with ``bg`` the backward
    reduction of that BN)."""
    C = native()
    N, K = w2d.shape
    M = y.numel() // N

    def run(name):
        part = None
        if name == "g1":
            if part_needed:
                part = torch.empty((2, N, C.conv1x1_mtiles(M)), dtype=torch.float32, device=y.device)
            if bg is not None:
                C.conv1x1_forward(x2, w2d, y, part, Hi, Wi, stride, add, add_mask, bg.x, bg.mask, bg.mean, bg.invstd,
                                  bg.scale, bg.shift)
            else:
                C.conv1x1_forward(x2, w2d, y, part, Hi, Wi, stride, add, add_mask)
            return part
        bm, bn, ns = _g2_parse(name)
        if part_needed:
            part = torch.empty((2, N, C.gemm2_mtiles(M, N, K, bm)), dtype=torch.float32, device=y.device)
        if bg is not None:
            C.gemm2_conv(x2, w2d, y, part, add, add_mask, Hi, Wi, stride, 1, 1, 0, bm, bn, bg.x, bg.mask, bg.mean,
                         bg.invstd, bg.scale, bg.shift, stages=ns, add_s2=add_s2)
        else:
            C.gemm2_conv(x2, w2d, y, part, add, add_mask, Hi, Wi, stride, 1, 1, 0, bm, bn, stages=ns, add_s2=add_s2)
        return part

    name = "g1"
    if _GEMM2 and K % 64 == 0 and N % 64 == 0:
        epi = (part_needed, add is not None, add_mask is not None, bg is not None and bg.mask is not None,
               bg is not None, add_s2)
        name = TUNER.pick(("1x1", M, K, N, stride, Hi, Wi, epi),
                          {n: (lambda n=n: run(n)) for n in ([] if add_s2 else ["g1"]) + _g2_names(N)})
    elif add_s2:
        raise RuntimeError("the compact stride-2 addend needs the gemm2 core")
    return run(name)


def _conv_wgrad(dy, x, dw, kh, kw, stride, pad):
    """fp32 weight gradient dw ([Cout, Cin] for 1x1, channels-last [Cout, Cin, KH, KW] for KxK) on
    the faster of the first core's split-M kernel and the LDS-DMA core (measured per shape)."""
    C = native()
    hi, wi = x.shape[2], x.shape[3]
    cout, cin = dy.shape[1], x.shape[1]
    if kh == kw == 1 and pad == 0:
        first = lambda: C.conv1x1_wgrad(dy, x, dw.view(cout, cin), hi, wi, stride)  # noqa: E731
    else:
        first = lambda: C.conv_wgrad(dy, x, dw, kh, kw, stride, pad)  # noqa: E731
    def mio():  # MIOpen's bf16 weight gradient (the 64-channel KxK layers' previous route)
        w = torch.empty((cout, cin, kh, kw), dtype=torch.bfloat16, device=dy.device)
        g = torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                                                [False, True, False])[1]
        dw.copy_(g)

    name = "w2"
    if _GEMM2 and cout % 64 == 0 and cin % 64 == 0:
        cands = {"w2": first}
        # gemm2.hip k_wgrad tilings (Cout x Cin*taps outputs): 0 128x128 (4 waves), 1 256x128
        # (4 waves), 2 256x256 (8 waves), 3 128x256 / 4 256x128 (8 waves of 64x64)
        ok = {0: True, 1: cout % 256 == 0 and cin % 128 == 0, 2: cout % 256 == 0 and cin % 256 == 0,
              3: cout % 128 == 0 and cin % 256 == 0, 4: cout % 256 == 0 and cin % 128 == 0}
        # 5 / 6: 64-channel KxK layers, two taps per 128-wide tile (K padded): 2 / 4 waves
        ok[5] = ok[6] = cin == 64 and kh * kw > 1
        for cfg in (0, 1, 2, 3, 4, 5, 6):
            if ok[cfg]:
                # LDS stages (3 do not fit 256x256; 4 = 32-row k-half units, see gemm2.hip)
                for ns in ((2, 3) if cfg != 2 else (2, 4)) + ((4,) if cfg == 0 else ()):
                    cands[f"w3_{cfg}" + ("" if ns == 2 else f"s{ns}")] = (
                        lambda cfg=cfg, ns=ns: C.gemm2_wgrad(dy, x, dw, kh, kw, stride, pad, hi, wi, cfg, ns))
        # (fewer, longer M slabs -- gemm2_wgrad sdiv=2, half the fp32 slab traffic -- measured: no
        # shape faster by more than 1 %, profiles/r3b/tuner_sdiv.json; not a candidate)
        if kh > 1 and cin < 128 and _MIOPEN_WGRAD:
            cands["miopen"] = mio
        name = TUNER.pick(("wgrad", tuple(x.shape), cout, kh, kw, stride, pad), cands)
    if name.startswith("w3"):
        sdiv = int(name.split("d")[1]) if "d" in name else 1
        C.gemm2_wgrad(dy, x, dw, kh, kw, stride, pad, hi, wi, int(name[3]), int(name[5]) if len(name) > 4 else 2,
                      sdiv=sdiv)
    elif name == "miopen":
        mio()
    else:
        first()


def _convkxk_gemm(x, w, stride, pad, stats: bool, bg=None):
    """KxK conv forward (channels-last bf16) on the fastest of {gemm2 implicit GEMM tiles, MIOpen}
    for this shape; returns (y, part or None) -- part: the following BN's statistics partials
    when the GEMM ran (MIOpen gives none), or with ``bg`` (a BNGradTap; y is then the gradient of
    that BN's output, e.g. a stride-1 input gradient run as a forward conv) the BN's backward
    reduction from the epilogue."""
    C = native()
    n, cin, h, wd = x.shape
    cout, k = w.shape[0], w.shape[2]
    ho, wo = (h + 2 * pad - k) // stride + 1, (wd + 2 * pad - k) // stride + 1
    y = torch.empty((n, cout, ho, wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    mio = lambda: torch.ops.aten.convolution(x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)  # noqa: E731

    def run(name):
        if name == "miopen":
            return mio(), None
        bm, bn, ns = _g2_parse(name)
        part = None
        if stats or bg is not None:
            part = torch.empty((2, cout, C.gemm2_mtiles(n * ho * wo, cout, k * k * cin, bm)), dtype=torch.float32,
                               device=x.device)
        if bg is not None:
            C.gemm2_conv(x, w, y, part, None, None, h, wd, stride, k, k, pad, bm, bn, bg.x, bg.mask, bg.mean,
                         bg.invstd, bg.scale, bg.shift, stages=ns)
        else:
            C.gemm2_conv(x, w, y, part, None, None, h, wd, stride, k, k, pad, bm, bn, stages=ns)
        return y, part

    def timed(name):
        # what the choice costs the step: with ``stats`` MIOpen leaves the following BN a
        # statistics pass over y (reduce + finalize), the GEMM leaves it a finalize of its partials;
        # with ``bg`` MIOpen leaves that BN's backward its reduction pass over (y, bn x)
        yy, part = run(name)
        if stats:
            v = [torch.empty(cout, dtype=torch.float32, device=x.device) for _ in range(6)]
            if part is None:
                C.bn_forward_stats(yy, v[0], v[1], None, None, v[2], v[3], v[4], v[5], cout, 1e-5, 0.1)
            else:
                C.bn_finalize_partials(part, part.shape[2], n * ho * wo, v[0], v[1], None, None, v[2], v[3], v[4],
                                       v[5], cout, 1e-5, 0.1)
        if bg is not None:
            mode = MASK_BITS if bg.mask is not None else MASK_X
            dx, dgw, dgb = torch.empty_like(yy), torch.empty_like(bg.scale), torch.empty_like(bg.scale)
            if part is None:
                C.bn_backward(yy, bg.x, None, mode, bg.scale, bg.mean, bg.invstd, bg.scale, bg.shift, dx, None,
                              dgw, dgb, cout, bg.mask)
            else:
                C.bn_backward_partials(part, part.shape[2], yy, bg.x, mode, bg.scale, bg.mean, bg.invstd, bg.scale,
                                       bg.shift, dx, None, dgw, dgb, cout, bg.mask)

    name = "miopen"
    if _GEMM2 and cin % 64 == 0 and cout % 64 == 0:
        epi = (stats, None if bg is None else bg.mask is not None)
        name = TUNER.pick(("kxk", n, cin, h, wd, cout, k, stride, pad, epi),
                          {nm: (lambda nm=nm: timed(nm)) for nm in ["miopen"] + _g2_names(cout)})
    return run(name)


def _dgrad_s2(dy, x, w, wf, bg=None):
    """Input gradient of a stride-2 3x3 / pad-1 conv: the fastest of MIOpen's backward-data and the
    gemm2 output-parity GEMMs (gemm2_dgrad_s2) per shape, the latter with the backward reduction of
    the BN whose output x is (``bg``, BNGradTap) in its epilogue -- timed with what each leaves that
    BN's backward.  Returns (dx, part or None)."""
    C = native()
    n, cin, h, wd = x.shape
    cout = dy.shape[1]

    def mio():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0], None

    def run(name):
        if name == "miopen":
            return mio()
        bm, bn, _ = _g2_parse(name)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        if bg is not None:
            part = C.gemm2_dgrad_s2(dy, wf, dx, bm, bn, bg.x, bg.mask, bg.mean, bg.invstd, bg.scale, bg.shift)
            return dx, part
        C.gemm2_dgrad_s2(dy, wf, dx, bm, bn)
        return dx, None

    def timed(name):
        dx, part = run(name)
        if bg is not None:
            mode = MASK_BITS if bg.mask is not None else MASK_X
            d2, dgw, dgb = torch.empty_like(dx), torch.empty_like(bg.scale), torch.empty_like(bg.scale)
            if part is None:
                C.bn_backward(dx, bg.x, None, mode, bg.scale, bg.mean, bg.invstd, bg.scale, bg.shift, d2, None, dgw,
                              dgb, cin, bg.mask)
            else:
                C.bn_backward_partials(part, part.shape[2], dx, bg.x, mode, bg.scale, bg.mean, bg.invstd, bg.scale,
                                       bg.shift, d2, None, dgw, dgb, cin, bg.mask)

    names = ["miopen"] + [nm for nm in ("g2_128x128", "g2_256x256", "g2_128x64", "g2_256x64") if cin % _g2_parse(nm)[1] == 0]
    name = TUNER.pick(("dgrad_s2", n, cin, h, wd, cout, None if bg is None else bg.mask is not None),
                      {nm: (lambda nm=nm: timed(nm)) for nm in names})
    return run(name)


def _conv_pro_fwd(x, w, stride, pad, scale, shift):
    """conv(relu(x * scale + shift)) (channels-last bf16 x = a BN's input; 1x1 or KxK) on gemm2 with
    the BN + ReLU applied to the A tile in LDS (kPro) and the following BN's statistics in the
    epilogue; the fastest 2-stage tile per shape.  Returns (y, part)."""
    C = native()
    n, cin, h, wd = x.shape
    cout, k = w.shape[0], w.shape[2]
    ho, wo = (h + 2 * pad - k) // stride + 1, (wd + 2 * pad - k) // stride + 1
    y = torch.empty((n, cout, ho, wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    w2 = w.reshape(cout, cin) if k == 1 else w

    def run(name):
        bm, bn, _ = _g2_parse(name)
        part = torch.empty((2, cout, C.gemm2_mtiles(n * ho * wo, cout, k * k * cin, bm)), dtype=torch.float32,
                           device=x.device)
        C.gemm2_conv(x, w2, y, part, None, None, h, wd, stride, k, k, pad, bm, bn, pro_scale=scale, pro_shift=shift)
        return y, part

    names = [nm for nm in _g2_names(cout) if _g2_parse(nm)[2] == 2]
    name = TUNER.pick(("pro", n, cin, h, wd, cout, k, stride, pad), {nm: (lambda nm=nm: run(nm)) for nm in names})
    return run(name)


def _conv_wgrad_pro(dy, x, dw, kh, kw, stride, pad, scale, shift):
    """fp32 weight gradient of conv(relu(x * scale + shift)) on the gemm2 weight-gradient kernels
    with the BN + ReLU applied to the X tile in LDS (the BN output is never materialised)."""
    C = native()
    hi, wi = x.shape[2], x.shape[3]
    cout, cin = dy.shape[1], x.shape[1]
    ok = {0: True, 1: cout % 256 == 0 and cin % 128 == 0, 3: cout % 128 == 0 and cin % 256 == 0,
          4: cout % 256 == 0 and cin % 128 == 0, 5: cin == 64 and kh * kw > 1, 6: cin == 64 and kh * kw > 1}
    cands = {f"w3_{cfg}": (lambda cfg=cfg: C.gemm2_wgrad(dy, x, dw, kh, kw, stride, pad, hi, wi, cfg, 2, scale, shift))
             for cfg, v in ok.items() if v}
    name = TUNER.pick(("wgrad_pro", tuple(x.shape), cout, kh, kw, stride, pad), cands)
    cands[name]()


class _BNReluConv(torch.autograd.Function):
    """conv(relu(bn(x))) for a training BatchNorm whose output only feeds this conv (ResNet bn1 ->
    conv2, bn2 -> conv3), the BN's statistics from its producer's epilogue (``part``): finalize,
    then the conv GEMM reading x with the BN + ReLU applied to each staged A tile in LDS (gemm2
    kPro), the next BN's statistics in its epilogue.  The BN output is never written or re-read.
    Backward: the input-gradient GEMM with this BN's backward reduction in its epilogue (relu'
    recomputed from x), the BN backward apply, and the weight gradient with the same BN + ReLU on
    its X tiles."""

    @staticmethod
    def forward(ctx, x, part, bn_w, bn_b, running_mean, running_var, eps, momentum, w_master, stride, pad):
        w = bf16_weight(w_master)
        if w.dim() == 4 and w.shape[2] > 1:
            w = w.contiguous(memory_format=torch.channels_last)
        ctx.wdtype = w_master.dtype
        ctx.wparam = w_master
        ctx.set_materialize_grads(False)
        ctx.wt = _TSHADOWS.get(w_master.data_ptr()) if w_master.dtype == torch.float32 else None
        n, c, h, wd = x.shape
        f32 = dict(dtype=torch.float32, device=x.device)
        mean, invstd, scale, shift = (torch.empty(c, **f32) for _ in range(4))
        native().bn_finalize_partials(part, part.shape[2], n * h * wd, bn_w, bn_b, running_mean, running_var, mean,
                                      invstd, scale, shift, c, float(eps), float(momentum))
        y, part_out = _conv_pro_fwd(x, w, stride, pad, scale, shift)
        ctx.geom = (stride, pad)
        ctx.save_for_backward(x, w, bn_w, mean, invstd, scale, shift)
        ctx.mark_non_differentiable(part_out)
        return y, part_out

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w, bn_w, mean, invstd, scale, shift = ctx.saved_tensors
        if dy is None:
            ctx.wparam = None
            return (None,) * 11
        s, p = ctx.geom
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, c, h, wd = x.shape
        cout, k = w.shape[0], w.shape[2]
        dw = None
        if ctx.needs_input_grad[8]:
            # the weight gradient first, on the weight-gradient side stream (as _Conv1x1 /
            # _ConvKxK), beside the input-gradient / BN-backward chain below
            def wg():
                d = torch.empty(w.shape, dtype=torch.float32, device=w.device,
                                memory_format=torch.channels_last if k > 1 else torch.contiguous_format)
                _conv_wgrad_pro(dy, x, d, k, k, s, p, scale, shift)
                return d if ctx.wdtype == torch.float32 else d.to(ctx.wdtype)

            dw = _on_wgrad_stream(ctx.wparam, (dy, x, scale, shift), wg)
        ctx.wparam = None
        bg = BNGradTap(x, None, mean, invstd, scale, shift)
        # gradient of the (never materialised) BN output, with that BN's backward reduction
        if k == 1:
            wt = ctx.wt if ctx.wt is not None else w.reshape(cout, c).t().contiguous()
            dbn = torch.empty_like(x, memory_format=torch.channels_last)
            part = _conv1x1_gemm(dy, wt, dbn, h, wd, 1, True, None, None, bg)
        else:
            wf = ctx.wt if ctx.wt is not None and ctx.wt.dim() == 4 else None  # rot180(W)^T shadow
            if wf is None:
                wf = torch.flip(w, (2, 3)).transpose(0, 1).contiguous(memory_format=torch.channels_last)
            if s == 1:
                dbn, part = _convkxk_gemm(dy, wf, 1, p, False, bg)
            else:
                dbn, part = _dgrad_s2(dy, x, w, wf, bg)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dgw, dgb = torch.empty_like(bn_w), torch.empty_like(bn_w)
        if part is not None:
            native().bn_backward_partials(part, part.shape[2], dbn, x, MASK_X, bn_w, mean, invstd, scale, shift, dx,
                                          None, dgw, dgb, c, None)
        else:
            native().bn_backward(dbn, x, None, MASK_X, bn_w, mean, invstd, scale, shift, dx, None, dgw, dgb, c, None)
        return dx, None, dgw, dgb, None, None, None, None, dw, None, None


def bn_relu_conv_ok(bn, conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Can _BNReluConv run conv(relu(bn(x))) (x: the BN's bf16 channels-last input)?"""
    if not (_GEMM2 and bn.training and getattr(bn, "relu", False) and bn._fast_ok(x, None) and conv.training):
        return False
    k, st, pd = conv.kernel_size, conv.stride, conv.padding
    if k[0] != k[1] or st[0] != st[1] or pd[0] != pd[1] or conv.groups != 1 or conv.bias is not None:
        return False
    if conv.dilation != (1, 1) or conv.padding_mode != "zeros" or k[0] not in (1, 3):
        return False
    if k[0] == 1 and (pd[0] != 0 or st[0] != 1):
        return False
    if k[0] == 3 and (pd[0] != 1 or st[0] not in (1, 2)):
        return False
    w = conv.weight
    return (conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and bn.weight.dtype == torch.float32 and
            (k[0] == 1 or w.is_contiguous(memory_format=torch.channels_last)))


def bn_relu_conv(bn, conv: nn.Conv2d, x, part):
    """(conv(relu(bn(x))), the next BN's statistics partials) on _BNReluConv (callers check
    bn_relu_conv_ok; ``part``: bn's statistics partials from x's producer)."""
    bn._nbt_pending += 1
    return _BNReluConv.apply(x, part, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum,
                             conv.weight, conv.stride[0], conv.padding[0])


def bn_pro_pays(bn, conv: nn.Conv2d, x, part) -> bool:
    """Should conv(relu(bn(x))) for a 1x1 ``conv`` run with the BN applied in the GEMM's operand
    prologue (_BNReluConv) rather than as its own apply pass?  Measured per layer shape, once (like
    every tuner pick), on the real operands: the apply pass (finalize + BN + ReLU, output written)
    + the tuned plain GEMM + the tuned weight gradient against the finalize + the prologue GEMM +
    the prologue weight gradient (the BN output never written, but every A / X tile transformed in
    LDS).  Globally the two were a wash (profiles/ab_r2/prologue_*: -0.23 ms of apply passes,
    +0.10..0.17 ms of GEMM), so the choice is made layer by layer (``tools/tuner_dump.py`` lists
    it under the key 'bnpro')."""
    if not _BN_PRO_TUNE or part is None or conv.kernel_size != (1, 1) or not bn_relu_conv_ok(bn, conv, x):
        return False
    n, c, h, wd = x.shape
    cout = conv.out_channels
    key = ("bnpro", n, c, h, wd, cout)
    got = TUNER.cache.get(key)
    if got is None:
        C = native()
        cl = torch.channels_last
        w = bf16_weight(conv.weight)
        w2 = w.reshape(cout, c)
        f32 = dict(dtype=torch.float32, device=x.device)
        rm, rv = bn.running_mean.clone(), bn.running_var.clone()  # (the real buffers stay untouched)
        mean, invstd, scale, shift = (torch.empty(c, **f32) for _ in range(4))
        y = torch.empty_like(x, memory_format=cl)
        out = torch.empty((n, cout, h, wd), dtype=torch.bfloat16, device=x.device, memory_format=cl)
        dy = torch.randn((n, cout, h, wd), device=x.device).to(torch.bfloat16).contiguous(memory_format=cl)
        dw = torch.empty((cout, c), **f32)
        eps, mom = float(bn.eps), float(bn.momentum)

        def apply():
            C.bn_forward_partials(part, part.shape[2], x, None, y, bn.weight, bn.bias, rm, rv, mean, invstd, scale,
                                  shift, c, eps, mom, True, None)
            _conv1x1_gemm(y, w2, out, h, wd, 1, True)
            _conv_wgrad(dy, y, dw, 1, 1, 1, 0)

        def pro():
            C.bn_finalize_partials(part, part.shape[2], n * h * wd, bn.weight, bn.bias, rm, rv, mean, invstd, scale,
                                   shift, c, eps, mom)
            _conv_pro_fwd(x, w, 1, 0, scale, shift)
            _conv_wgrad_pro(dy, x, dw, 1, 1, 1, 0, scale, shift)

        got = TUNER.pick(key, {"apply": apply, "pro": pro})
    return got == "pro"


class ResidualTap:
    """Hands a fused BN's residual gradient to the stride-1 1x1 conv that reads the same block
    input (ResNet identity blocks: x feeds conv1 and is bn3's residual).  bn3's backward stores
    its (dy, ReLU bits) here instead of writing a dres tensor; conv1's backward -- which autograd
    always runs later, since it needs the gradient that flows down from bn3 through conv3, bn2,
    conv2 and bn1 -- adds dy * bits in its dgrad GEMM epilogue.  That removes one full-size write
    (dres) and the autograd add kernel (read 2, write 1) per identity block."""

    __slots__ = ("armed", "dy", "mask")

    def __init__(self):
        self.armed = False  # set when conv1 took the MFMA path (its backward will consume the tap)
        self.dy = None
        self.mask = None

    def take(self):
        dy, mask = self.dy, self.mask
        self.dy = self.mask = None
        return dy, mask


class BNGradTap:
    """Lets the 1x1 conv that consumes a fused BN's output compute that BN's backward reduction
    (sum dz, sum dz * x-hat per channel) in its dgrad epilogue, on the gradient tile it has just
    produced (gemm.hip BnBwdTap) -- the BN backward then skips its reduction pass over dy and x.
    Valid only when the conv's input gradient IS the complete gradient of the BN output: the
    model opts in (conv_bn(..., bn_grad=True)) where the BN output has no other consumer, or its
    other gradient paths are summed into the same epilogue (ResidualTap / alias)."""

    __slots__ = ("x", "mask", "mean", "invstd", "scale", "shift", "part")

    def __init__(self, x, mask, mean, invstd, scale, shift):
        self.x, self.mask, self.mean, self.invstd, self.scale, self.shift = x, mask, mean, invstd, scale, shift
        self.part = None


class S2Tap:
    """Hands the input gradient of a stride-2 1x1 conv (a ResNet downsample) to the stride-1 1x1
    conv that reads the same tensor (the block's conv1, through the alias it returned).  The
    downsample's backward computes only the compact gradient [img, C, ceil(H/2), ceil(W/2)] (a
    plain GEMM over its output rows) and returns no gradient for the alias; conv1's backward --
    which autograd runs after it, the alias being one of conv1's outputs -- adds it on the even
    (h, w) rows in its dgrad epilogue (gemm2 kAddS2).  No zero-filled full-size gradient is
    written or re-read (MIOpen's strided backward-data writes one: zero fill + scatter)."""

    __slots__ = ("dx",)

    def __init__(self):
        self.dx = None


_SHADOWS: list = []  # [fp32 flat param buffer, bf16 shadow] pairs (FlatStore.enable_bf16_shadow)


def register_weight_shadow(flat: torch.Tensor, shadow: torch.Tensor):
    _SHADOWS.append((flat, shadow))


def unregister_weight_shadow(shadow: torch.Tensor):
    _SHADOWS[:] = [(f, s) for f, s in _SHADOWS if s is not shadow]


# fp32 conv weight data_ptr -> bf16 backward operand (FlatStore tshadow): [Cin, Cout] for 1x1,
# rot180(W)^T as a channels-last [Cin, Cout, KH, KW] for KxK
_TSHADOWS: dict = {}


def register_transposed_weight(p: torch.Tensor, view: torch.Tensor):
    _TSHADOWS[p.data_ptr()] = view


def mark_transposed_reader(*params) -> None:
    """Ask the optimizer's flat store for a bf16 W^T copy of these Linear weights, refreshed with the
    shadow (one transpose-cast kernel per step for all of them): the gemm2 input-gradient GEMMs
    with an epilogue (GELU backward, a residual gradient) read it as their B operand."""
    if not (_GELU_MLP or _RES_LINK):
        return
    for p in params:
        if p is not None and p.dim() == 2:
            p.reads_bf16_shadow_t = True


def transposed_weight(w: torch.Tensor):
    """The registered bf16 W^T of fp32 weight ``w`` (mark_transposed_reader), or None."""
    t = _TSHADOWS.get(w.data_ptr())
    return t if t is not None and w.dim() == 2 and tuple(t.shape) == (w.shape[1], w.shape[0]) else None


def unregister_transposed_weight(p: torch.Tensor):
    _TSHADOWS.pop(p.data_ptr(), None)


# Host work that may run whenever the forward is ahead of the GPU (e.g. the engine dropping the
# previous steps' gathered gradients, ~2 us per tensor): bf16_weight runs each task once per conv
# of the forward, where the host leads the GPU by milliseconds, instead of at the step boundary or
# the start of backward, where a late host idles the GPU.
_HOST_IDLE_TASKS: list = []


def add_host_idle_task(fn) -> None:
    _HOST_IDLE_TASKS.append(fn)


def remove_host_idle_task(fn) -> None:
    try:
        _HOST_IDLE_TASKS.remove(fn)
    except ValueError:
        pass


def bf16_weight(w: torch.Tensor, idle: bool = True) -> torch.Tensor:
    """The bf16 view of fp32 master weight ``w`` in a registered shadow (same shape and strides),
    else a fresh cast.  The shadow is refreshed by the optimizer with one cast kernel per step, so
    a ResNet-50 forward reads its 53 conv weights without 53 autocast cast launches.  ``idle``:
    run the registered host idle tasks first (forward: the host leads the GPU there; a backward
    caller passes False -- at the start of backward the GPU waits for the host)."""
    if idle:
        for fn in _HOST_IDLE_TASKS:
            fn()
    if w.dtype == torch.bfloat16:
        return w
    p = w.data_ptr()
    for flat, sh in _SHADOWS:
        base = flat.data_ptr()
        if base <= p < base + flat.numel() * 4 and w.device == flat.device:
            return sh.as_strided(w.shape, w.stride(), (p - base) // 4)
    return w.to(torch.bfloat16)


def has_weight_shadow(w: torch.Tensor) -> bool:
    """Is fp32 parameter ``w`` inside a registered bf16 shadow (bf16_weight returns a view)?"""
    if w.dtype != torch.float32 or not w.is_cuda:
        return False
    p = w.data_ptr()
    return any(flat.data_ptr() <= p < flat.data_ptr() + flat.numel() * 4 and w.device == flat.device
               for flat, _ in _SHADOWS)


class _ShadowLinear(torch.autograd.Function):
    """y = x W^T + b under bf16 autocast for an fp32 master weight with a bf16 shadow: the GEMM
    reads the shadow (refreshed once per step by the optimizer) instead of autocast casting W
    every forward, and the backward writes dW in fp32 straight from the GEMM (hipBLASLt
    ``mm(..., out_dtype=float32)``) instead of a bf16 dW plus a cast kernel into the fp32 grad.
    BERT-base spent ~3 ms of a 38.8 ms step in those casts (profiles/r4/r4n/)."""

    @staticmethod
    def forward(ctx, x, w_master, bias, residual=None, link=None):
        dt = torch.bfloat16
        w = bf16_weight(w_master)
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype != dt:
            x2 = x2.to(dt)
        r2 = None if residual is None else residual.reshape(-1, w.shape[0])
        y = _linear_fwd(x2, w, bias, r2)
        ctx.save_for_backward(x2, w_master)
        ctx.has_bias = bias is not None
        ctx.xshape, ctx.xdtype = x.shape, x.dtype
        ctx.rshape = None if residual is None else residual.shape
        # ResidualLink: the consumer side (this Linear reads x, a later one adds x as its residual)
        # arms the link; the residual side hands its gradient over instead of returning it
        ctx.link_in = ctx.link_out = None
        if link is not None and _RES_LINK:
            if residual is None and x.dtype == dt and x.dim() >= 2:
                link.armed, link.x = True, x
                ctx.link_in = link
            elif residual is not None and link.armed and link.x is residual:
                ctx.link_out = link
                link.armed, link.x = False, None
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w_master = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != torch.bfloat16:
            dy2 = dy2.to(torch.bfloat16)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            g = ctx.link_in.take() if ctx.link_in is not None else None
            if g is not None:
                # the residual's gradient (handed over by the Linear that added x) joins in the GEMM
                dx = _dgrad(dy2, w_master, g.reshape(dy2.shape[0], -1)).view(ctx.xshape)
            else:
                dx = torch.mm(dy2, bf16_weight(w_master, idle=False)).view(ctx.xshape)
            if dx.dtype != ctx.xdtype:
                dx = dx.to(ctx.xdtype)
        if ctx.needs_input_grad[1]:
            # (on the caller's stream: a linear weight may be used twice in a graph -- a tied
            # decoder, a reused module -- and autograd sums such contributions on this stream)
            dw = _linear_wgrad(dy2, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum_f32(dy2)
        dres = dy.reshape(ctx.rshape) if ctx.rshape is not None and ctx.needs_input_grad[3] else None
        if dres is not None and ctx.link_out is not None:
            ctx.link_out.give(dres if dres.dtype == torch.bfloat16 else dres.to(torch.bfloat16))
            dres = None
        return dx, dw, db, dres, None


class ResidualLink:
    """Pairs the Linear that reads x with the later Linear that adds x back as its residual
    (BERT: qkv(x) ... attn_out(a, residual=x)), so x's two gradients meet in ONE GEMM: the
    residual side's backward (which runs first) hands dy over, and the reader's input gradient is
    addmm(dy, d_out, W) instead of mm + an autograd add.  The reader's forward arms the link (its
    _ShadowLinear path only, for the same tensor); a residual side that finds it unarmed returns its
    gradient normally.  One link per use, created in the forward."""

    __slots__ = ("armed", "x", "g")

    def __init__(self):
        self.armed, self.x, self.g = False, None, None

    def give(self, g):
        self.g = g if self.g is None else self.g + g

    def take(self):
        g, self.g = self.g, None
        return g


def _linear_fwd(x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
                res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x2 w^T (+ bias) (+ res) (bf16 [M, K] x [N, K] (+ bf16 [M, N]) -> [M, N]): per shape the
    faster of hipBLASLt (mm / addmm with the bf16 bias or the residual as C) and the hipps
    1x1-convolution GEMM cores (a Linear is a 1x1 convolution over M pixels; their kBias epilogue
    adds the fp32 master bias to the fp32 accumulator before the bf16 rounding, kAdd the residual
    in the same pass)."""
    M, K = x2.shape
    N = w.shape[0]
    if res is not None and res.dtype == torch.float32:
        # an fp32 residual stream (Llama: x + wo(a), x + w2(.)): one hipBLASLt GEMM with the fp32
        # residual as C and an fp32 output (aten addmm.dtype) instead of a bf16 GEMM output plus a
        # mixed-dtype add pass over the residual stream
        return torch.ops.aten.addmm.dtype(res, x2, w.t(), torch.float32)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x2.device)

    def blas():
        if res is not None:
            torch.addmm(res, x2, w.t(), out=y)
            if bias is not None:
                y.add_(bf16_weight(bias))
        elif bias is None:
            torch.mm(x2, w.t(), out=y)
        else:
            torch.addmm(bf16_weight(bias), x2, w.t(), out=y)

    if not (_GEMM2 and N % 64 == 0 and K % 64 == 0 and M >= 1024 and x2.is_contiguous() and w.is_contiguous()
            and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and y.data_ptr() % 16 == 0
            and (bias is None or (bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N))
            and (res is None or (res.dtype == torch.bfloat16 and res.is_contiguous() and res.data_ptr() % 16 == 0))):
        blas()
        return y
    C = native()
    cands = {"blas": blas}
    b = None if bias is None else bias.detach()
    for name in _g2_names(N):
        bm, bn, ns = _g2_parse(name)
        cands[name] = (lambda bm=bm, bn=bn, ns=ns:
                       C.gemm2_conv(x2, w, y, None, res, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns, bias=b))
    pick = TUNER.pick(("lfwd", M, N, K, bias is not None, res is not None), cands)
    cands[pick]()
    return y


def _linear_fwd_nobias(x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _linear_fwd(x2, w)


def _linear_wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """dW = dy2^T x2 in fp32 ([N, K] from bf16 [M, N] and [M, K]): the faster, per shape, of
    hipBLASLt (mm with an fp32 output) and the gemm2 split-M weight-gradient kernels (a Linear's
    dW is a 1x1 convolution's).  hipBLASLt picked 64x64 macro tiles for BERT-base's 768-wide
    dW GEMMs (M = 16384 tokens): 186 TFLOP/s (profiles/r4/r4n/)."""
    M, N = dy2.shape
    K = x2.shape[1]
    dw = torch.empty((N, K), dtype=torch.float32, device=dy2.device)

    def mm():
        torch.ops.aten.mm.dtype_out(dy2.t(), x2, torch.float32, out=dw)

    if not (_GEMM2 and N % 64 == 0 and K % 64 == 0 and M >= 1024 and dy2.is_contiguous() and x2.is_contiguous()
            and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0):
        mm()
        return dw
    C = native()
    cands = {"mm": mm}
    ok = {0: True, 1: N % 256 == 0 and K % 128 == 0, 2: N % 256 == 0 and K % 256 == 0,
          3: N % 128 == 0 and K % 256 == 0, 4: N % 256 == 0 and K % 128 == 0}
    for cfg in (0, 1, 2, 3, 4):
        if ok[cfg]:
            for ns in ((2, 3) if cfg != 2 else (2, 4)):
                cands[f"w3_{cfg}" + ("" if ns == 2 else f"s{ns}")] = (
                    lambda cfg=cfg, ns=ns: C.gemm2_wgrad(dy2, x2, dw, 1, 1, 1, 0, 1, 1, cfg, ns))
    name = TUNER.pick(("lwgrad", M, N, K), cands)
    cands[name]()
    return dw


def _g2_ok(*ts) -> bool:
    return all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts)


def _gelu_linear_fwd(x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor]):
    """(gelu(x2 w^T + bias), x2 w^T + bias), both bf16 [M, N]: per shape the faster of hipBLASLt
    addmm + PyTorch's GELU and the gemm2 kGelu epilogue (gemm2.hip: the pre-activation and the
    GELU written by the GEMM's own epilogue -- no GELU pass re-reading the pre-activation)."""
    M, K = x2.shape
    N = w.shape[0]
    pre = torch.empty((M, N), dtype=torch.bfloat16, device=x2.device)
    post = torch.empty_like(pre)

    def blas():
        if bias is None:
            torch.mm(x2, w.t(), out=pre)
        else:
            torch.addmm(bf16_weight(bias), x2, w.t(), out=pre)
        torch._C._nn.gelu(pre, out=post)

    if not (_GEMM2 and N % 64 == 0 and K % 64 == 0 and M >= 1024 and _g2_ok(x2, w)
            and (bias is None or (bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N))):
        blas()
        return post, pre
    C = native()
    b = None if bias is None else bias.detach()
    cands = {"blas": blas}
    for name in _g2_names(N):
        bm, bn, ns = _g2_parse(name)
        cands[name] = (lambda bm=bm, bn=bn, ns=ns:
                       C.gemm2_conv(x2, w, post, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns, bias=b,
                                    gelu_pre=pre, gelu=1))
    cands[TUNER.pick(("gelu_fwd", M, N, K, bias is not None), cands)]()
    return post, pre


def _gelu_dgrad(dy2: torch.Tensor, w: torch.Tensor, pre: torch.Tensor, wt=None, bias_grad: bool = False) -> torch.Tensor:
    """d pre = gelu'(pre) * (dy2 w) (bf16 [M, K] from dy2 [M, N], w [N, K]: the input gradient of
    the Linear after a GELU, through the GELU): per shape the faster of hipBLASLt mm + PyTorch's
    GELU backward and the gemm2 kGeluB epilogue over ``wt`` = w^T [K, N] (the flat store's
    transposed shadow, mark_transposed_reader; without one, no gemm2 candidate).  ``bias_grad``:
    the column sum of d pre (the first Linear's bias gradient) is left for colsum_f32 -- the gemm2
    epilogue sums its own output tiles (kGeluBS), so no pass re-reads d pre."""
    M, N = dy2.shape
    K = w.shape[1]

    def blas():
        out = torch.ops.aten.gelu_backward(torch.mm(dy2, w), pre)
        if bias_grad:
            stash_colsum(out, colsum_f32(out))
        return out

    if not (_GEMM2 and wt is not None and N % 64 == 0 and K % 64 == 0 and M >= 1024 and _g2_ok(dy2, wt, pre)):
        return blas()
    C = native()
    out = torch.empty((M, K), dtype=torch.bfloat16, device=dy2.device)

    def g2(bm, bn, ns):
        part = None
        if bias_grad:
            part = torch.empty((C.gemm2_mtiles(M, K, N, bm), K), dtype=torch.float32, device=dy2.device)
        C.gemm2_conv(dy2, wt, out, part, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns, gelu_pre=pre, gelu=2)
        if bias_grad:
            db = torch.empty(K, dtype=torch.float32, device=dy2.device)
            C.colsum_fold(part, db)
            stash_colsum(out, db)
        return out

    cands = {"blas": blas}
    for name in _g2_names(K):
        bm, bn, ns = _g2_parse(name)
        cands[name] = (lambda bm=bm, bn=bn, ns=ns: g2(bm, bn, ns))
    return cands[TUNER.pick(("gelu_dgrad", M, N, K, bias_grad), cands)]()


def _dgrad(dy2: torch.Tensor, w_master: torch.Tensor, add: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = dy2 W (+ add) in bf16 ([M, K] from dy2 [M, N] and the weight's [N, K] shadow; ``add``
    bf16 [M, K], a residual's gradient): hipBLASLt (mm, or addmm with ``add`` as C -- which
    PyTorch first copies into the output), or with a registered W^T (mark_transposed_reader) the
    gemm2 tiles with ``add`` in the kAdd epilogue, the faster per shape."""
    w = bf16_weight(w_master, idle=False)
    M, N = dy2.shape
    K = w.shape[1]

    def blas():
        return torch.mm(dy2, w) if add is None else torch.addmm(add, dy2, w)

    wt = transposed_weight(w_master)
    if not (_GEMM2 and wt is not None and add is not None and N % 64 == 0 and K % 64 == 0 and M >= 1024
            and add.dtype == torch.bfloat16 and tuple(add.shape) == (M, K) and _g2_ok(dy2, wt, add)):
        return blas()
    C = native()
    out = torch.empty((M, K), dtype=torch.bfloat16, device=dy2.device)

    def g2(bm, bn, ns):
        C.gemm2_conv(dy2, wt, out, None, add, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns)
        return out

    cands = {"blas": blas}
    for name in _g2_names(K):
        bm, bn, ns = _g2_parse(name)
        cands[name] = (lambda bm=bm, bn=bn, ns=ns: g2(bm, bn, ns))
    return cands[TUNER.pick(("dgrad_add", M, N, K), cands)]()


class _GeluMLP(torch.autograd.Function):
    """y = gelu(x W1^T + b1) W2^T + b2 (+ x): a transformer MLP (BERT's intermediate / output
    Linear pair, exact-erf GELU, optionally with its own input as the residual) as ONE autograd
    node on the bf16 weight shadows (see _ShadowLinear):

    * forward: the first GEMM writes the pre-activation AND the GELU in its epilogue
      (_gelu_linear_fwd), the second adds b2 and the residual in its own (_linear_fwd);
    * backward: the second Linear's input gradient carries the GELU backward in its epilogue
      (_gelu_dgrad), and with the residual the first Linear's input gradient is one hipBLASLt
      addmm with dy as C -- the residual's gradient joins there instead of in an autograd add.

    Same math as hnn.Linear -> F.gelu -> hnn.Linear(residual=x) (which hipps.models used before)."""

    @staticmethod
    def forward(ctx, x, w1m, b1, w2m, b2, res_x):
        dt = torch.bfloat16
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype != dt:
            x2 = x2.to(dt)
        post, pre = _gelu_linear_fwd(x2, bf16_weight(w1m), b1)
        w2 = bf16_weight(w2m)
        y = _linear_fwd(post, w2, b2, x2 if res_x else None)
        ctx.save_for_backward(x2, pre, post, w1m, w2m)
        ctx.has_b1, ctx.has_b2, ctx.res_x = b1 is not None, b2 is not None, bool(res_x)
        ctx.xshape, ctx.xdtype = x.shape, x.dtype
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, pre, post, w1m, w2m = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != torch.bfloat16:
            dy2 = dy2.to(torch.bfloat16)
        dy2 = dy2.contiguous()
        dpre = _gelu_dgrad(dy2, bf16_weight(w2m, idle=False), pre, transposed_weight(w2m),
                           bias_grad=ctx.has_b1 and ctx.needs_input_grad[2])
        dx = dw1 = db1 = dw2 = db2 = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad(dpre, w1m, dy2 if ctx.res_x else None).view(ctx.xshape)
            if dx.dtype != ctx.xdtype:
                dx = dx.to(ctx.xdtype)
        if ctx.needs_input_grad[3]:
            dw2 = _linear_wgrad(dy2, post)
        if ctx.has_b2 and ctx.needs_input_grad[4]:
            db2 = colsum_f32(dy2)
        if ctx.needs_input_grad[1]:
            dw1 = _linear_wgrad(dpre, x2)
        if ctx.has_b1 and ctx.needs_input_grad[2]:
            db1 = colsum_f32(dpre)
        return dx, dw1, db1, dw2, db2, None


def gelu_mlp(x: torch.Tensor, l1: nn.Linear, l2: nn.Linear, residual_x: bool = False) -> torch.Tensor:
    """l2(gelu(l1(x))) (+ x with ``residual_x``): one _GeluMLP node under bf16 autocast when weight
    shadows cover both Linears (the fused GEMM epilogues), the module composition otherwise."""
    if (_GELU_MLP and _SHADOW_LINEAR and shadow_linear_ok(x, l1.weight, l1.bias) and shadow_linear_ok(x, l2.weight, l2.bias)
            and x.shape[-1] == l1.weight.shape[1] and l2.weight.shape[1] == l1.weight.shape[0]
            and (not residual_x or (l2.weight.shape[0] == x.shape[-1] and x.dtype == torch.bfloat16))):
        return _GeluMLP.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, residual_x)
    h = F.gelu(l1(x))
    return l2(h, residual=x) if residual_x and isinstance(l2, Linear) else (l2(h) + x if residual_x else l2(h))


# column sums computed as a by-product of the kernel that wrote a gradient (LayerNorm backward
# over its dx: the bias gradient of the Linear before it), keyed by data pointer; each entry holds
# its tensor (the pointer cannot be reused while it waits) and the tensor's version (an in-place
# change voids it).  Bounded: an entry nobody consumes is dropped after 4 newer ones.
_COLSUM_STASH: "collections.OrderedDict" = collections.OrderedDict()


def stash_colsum(t: torch.Tensor, cs: torch.Tensor) -> None:
    """Record cs = t.reshape(-1, t.shape[-1]).sum(0) (fp32) for colsum_f32 to return for t."""
    _COLSUM_STASH[t.data_ptr()] = (t, t._version, cs)
    while len(_COLSUM_STASH) > 4:
        _COLSUM_STASH.popitem(last=False)


def colsum_f32(t: torch.Tensor) -> torch.Tensor:
    """t.sum(0) in fp32 for a 2-d bf16 device tensor (csrc/xent.hip k_colsum: deterministic,
    ~4x PyTorch's reduce on a bias gradient); torch.sum otherwise.  A sum the producing kernel
    already computed (stash_colsum) is returned without a pass over t."""
    if _COLSUM_STASH and t.dim() == 2:
        hit = _COLSUM_STASH.pop(t.data_ptr(), None)
        if hit is not None:
            src, ver, cs = hit
            if (src._version == ver and src.dtype == t.dtype and src.numel() == t.numel()
                    and src.shape[-1] == t.shape[1] and src.is_contiguous() and t.is_contiguous()):
                return cs
    if (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.is_contiguous() and t.shape[1] % 8 == 0
            and t.data_ptr() % 16 == 0):
        out = torch.empty(t.shape[1], dtype=torch.float32, device=t.device)
        native().colsum_bf16(t, out)
        return out
    return torch.sum(t, 0, dtype=torch.float32)


def mark_shadow_reader(*params) -> None:
    """Tag parameters read through bf16_weight by hipps ops other than the conv kernels (whose
    4-D weights the optimizer recognises by shape): bf16_weights='auto' then keeps a shadow."""
    for p in params:
        if p is not None:
            p.reads_bf16_shadow = True


def shadow_linear_ok(x: torch.Tensor, weight: torch.Tensor, bias=None, residual=None) -> bool:
    return (_SHADOW_LINEAR and x.is_cuda and torch.is_autocast_enabled() and
            torch.get_autocast_dtype("cuda") == torch.bfloat16 and has_weight_shadow(weight) and
            (bias is None or has_weight_shadow(bias)) and
            (residual is None or (residual.dtype in (torch.bfloat16, torch.float32) and residual.shape[-1] == weight.shape[0]
                                  and residual.numel() == x.numel() // x.shape[-1] * weight.shape[0]
                                  and (residual.dtype == torch.bfloat16 or (bias is None and residual.is_contiguous())))))


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, residual=None, link=None) -> torch.Tensor:
    """F.linear (+ residual), on the bf16 weight shadow when one covers ``weight`` (see
    _ShadowLinear; a bf16 residual is added in the GEMM's epilogue or as hipBLASLt's C).
    ``link``: a ResidualLink shared with the Linear that reads (or adds) the same x."""
    if residual is not None and not _LINEAR_RESIDUAL:
        return residual + linear(x, weight, bias)
    if shadow_linear_ok(x, weight, bias, residual):
        return _ShadowLinear.apply(x, weight, bias, residual, link)
    y = F.linear(x, weight, bias)
    return y if residual is None else residual + y


class Linear(nn.Linear):
    """nn.Linear that reads the bf16 weight shadow under bf16 autocast (hipps.ops.nn.linear).
    Its parameters carry ``reads_bf16_shadow`` so the optimizer's ``bf16_weights='auto'`` knows
    a reader exists."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        mark_shadow_reader(self.weight, self.bias)

    def forward(self, x, residual=None, link=None):
        return linear(x, self.weight, self.bias, residual, link)


class _CrossEntropy(torch.autograd.Function):
    """Mean softmax cross-entropy of bf16 logits [rows, vocab] (csrc/xent.hip): one read of the
    logits in the forward (online log-sum-exp), one read + one bf16 gradient write in the
    backward; no fp32 copy of the logits."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        # the mean runs over the rows that carry a loss: not ignore_index and inside [0, V) (an
        # out-of-range label contributes no loss -- F.cross_entropy raises on it -- and is not
        # counted either); every row ignored -> 0 / 0 = NaN, as F.cross_entropy returns.  Loss,
        # count and mean come out of two launches (k_xent_fwd, k_xent_mean).
        loss, n, lse = native().xent_forward(logits, labels, int(ignore_index))
        ctx.save_for_backward(logits, labels, lse, n)
        ctx.ignore = int(ignore_index)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, n = ctx.saved_tensors
        dx = torch.empty_like(logits)
        if g.dtype != torch.float32 or g.numel() != 1 or not g.is_contiguous():
            g = g.to(torch.float32).reshape(1).contiguous()
        native().xent_backward(logits, labels, lse, g, 1.0, ctx.ignore, dx, n)
        return dx, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """F.cross_entropy(logits.float(), labels, ignore_index=...) (mean over non-ignored rows) on
    the fused kernel for contiguous bf16 device logits [.., vocab]; the PyTorch route otherwise."""
    V = logits.shape[-1]
    if (_FUSED_XENT and logits.is_cuda and logits.dtype == torch.bfloat16 and labels.dtype == torch.int64
            and labels.numel() * V == logits.numel() and 0 < labels.numel() < (1 << 24) and V > 0):
        # (the kernel's row count limits; empty batches and larger ones take the PyTorch route)
        return _CrossEntropy.apply(logits.reshape(-1, V).contiguous(), labels.reshape(-1).contiguous(), ignore_index)
    return F.cross_entropy(logits.float().reshape(-1, V), labels.reshape(-1), ignore_index=ignore_index)


# ---------------------------------------------------------------------------------- attention
# flash attention on the hipps MFMA kernels (csrc/attn.hip) instead of PyTorch SDPA (whose ROCm
# route is aotriton, Triton-generated code); HIPPS_FUSED_ATTN=0 keeps SDPA for A/B runs
_FUSED_ATTN = _os.environ.get("HIPPS_FUSED_ATTN", "1") != "0"


def _attn_rows_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4 and t.stride(3) == 1
            and all(x % 8 == 0 for x in t.stride()[:3]) and t.data_ptr() % 16 == 0)


def attention_ok(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> bool:
    """Whether :func:`attention` runs on the hipps kernels for these operands."""
    return (_FUSED_ATTN and _attn_rows_ok(q) and _attn_rows_ok(k) and _attn_rows_ok(v) and q.shape[3] in (64, 128)
            and k.shape == v.shape and k.shape[3] == q.shape[3] and k.shape[0] == q.shape[0]
            and q.shape[2] % k.shape[2] == 0 and (not causal or q.shape[1] == k.shape[1])
            and 0 < q.shape[1] < (1 << 24) and 0 < k.shape[1] < (1 << 24))


class _FlashAttention(torch.autograd.Function):
    """o = softmax(q k^T * scale [+ causal / key-padding mask]) v on [B, S, H, D] bf16 operands
    (csrc/attn.hip): forward keeps only o and the per-row log-sum-exp; backward recomputes P in
    the dQ and the dK/dV kernels (deterministic: no float atomics)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, kv_len):
        o, lse = native().attn_forward(q, k, v, causal, scale, kv_len)
        ctx.save_for_backward(q, k, v, o, lse, kv_len)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kv_len = ctx.saved_tensors
        do = do.to(torch.bfloat16)
        if not _attn_rows_ok(do):
            do = do.contiguous()
        dq, dk, dv = native().attn_backward(do, q, k, v, o, lse, ctx.causal, ctx.scale, kv_len)
        return dq, dk, dv, None, None, None


class _FlashAttentionQKV(torch.autograd.Function):
    """Attention over q / k / v packed in one [B, S, 3, H, D] tensor (a fused QKV projection's
    output viewed per head).  The backward writes dq, dk and dv straight into ONE packed gradient
    of the same layout (attn_backward's strided outputs), so the projection's backward reads a
    single [B*S, 3*H*D] gradient -- no per-slice zero-fill / copy / sum that autograd would run for
    three separate views."""

    @staticmethod
    def forward(ctx, qkv, causal, scale, kv_len):
        q, k, v = qkv.unbind(2)
        o, lse = native().attn_forward(q, k, v, causal, scale, kv_len)
        ctx.save_for_backward(qkv, o, lse, kv_len)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kv_len = ctx.saved_tensors
        do = do.to(torch.bfloat16)
        if not _attn_rows_ok(do):
            do = do.contiguous()
        g = torch.empty(qkv.shape, dtype=torch.bfloat16, device=qkv.device)
        q, k, v = qkv.unbind(2)
        gq, gk, gv = g.unbind(2)
        native().attn_backward(do, q, k, v, o, lse, ctx.causal, ctx.scale, kv_len, gq, gk, gv)
        return g, None, None, None


def attention_qkv(qkv: torch.Tensor, causal: bool = False, scale: Optional[float] = None,
                  kv_len: Optional[torch.Tensor] = None) -> torch.Tensor:
    """:func:`attention` of q, k, v packed as ``qkv`` [B, S, 3, H, D] (e.g. ``linear(x, W_qkv)
    .view(B, S, 3, H, D)``); returns [B, S, H, D]."""
    q, k, v = qkv.unbind(2)
    if attention_ok(q, k, v, causal) and qkv.dtype == torch.bfloat16:
        sc = float(scale) if scale is not None else 1.0 / (qkv.shape[-1] ** 0.5)
        kl = None if kv_len is None else kv_len.to(device=qkv.device, dtype=torch.int32).contiguous()
        return _FlashAttentionQKV.apply(qkv, bool(causal), sc, kl)
    return attention(q, k, v, causal=causal, scale=scale, kv_len=kv_len)


class _RopeAttentionPacked(torch.autograd.Function):
    """Llama's attention from ONE packed projection y [B, S, (Hq + 2 Hkv) * D] (q | k | v column
    blocks): RoPE on q and k (csrc/act.hip k_rope, strided reads), causal GQA flash attention with v
    read in place.  The backward writes dq, dk and dv straight into one packed gradient of y's
    layout and rotates its q / k blocks back in place -- the fused projection's backward then
    runs one GEMM each way, with no per-slice zero-fill / copy / add that autograd would run for
    three views of y."""

    @staticmethod
    def forward(ctx, y, cos, sin, hq, hkv, causal, scale):
        B, S, W = y.shape
        D = W // (hq + 2 * hkv)
        y2 = y.view(B * S, W)
        q = torch.empty(B, S, hq, D, dtype=y.dtype, device=y.device)
        k = torch.empty(B, S, hkv, D, dtype=y.dtype, device=y.device)
        C = native()
        C.rope_apply(y2[:, :hq * D], q.view(B * S, hq * D), cos, sin, S, D, 1.0)
        C.rope_apply(y2[:, hq * D:(hq + hkv) * D], k.view(B * S, hkv * D), cos, sin, S, D, 1.0)
        v = y[:, :, (hq + hkv) * D:].view(B, S, hkv, D)
        o, lse = C.attn_forward(q, k, v, causal, scale, None)
        ctx.save_for_backward(q, k, y, o, lse, cos, sin)
        ctx.meta = (hq, hkv, D, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, y, o, lse, cos, sin = ctx.saved_tensors
        hq, hkv, D, causal, scale = ctx.meta
        B, S, W = y.shape
        do = do.to(torch.bfloat16)
        if not _attn_rows_ok(do):
            do = do.contiguous()
        g = torch.empty(B, S, W, dtype=torch.bfloat16, device=y.device)
        v = y[:, :, (hq + hkv) * D:].view(B, S, hkv, D)
        gq = g[:, :, :hq * D].view(B, S, hq, D)
        gk = g[:, :, hq * D:(hq + hkv) * D].view(B, S, hkv, D)
        gv = g[:, :, (hq + hkv) * D:].view(B, S, hkv, D)
        C = native()
        C.attn_backward(do, q, k, v, o, lse, causal, scale, None, gq, gk, gv)
        g2 = g.view(B * S, W)
        for a, b in ((0, hq * D), (hq * D, (hq + hkv) * D)):  # rotate back in place (the backward of RoPE)
            C.rope_apply(g2[:, a:b], g2[:, a:b], cos, sin, S, D, -1.0)
        return g, None, None, None, None, None, None


def rope_attention_packed_ok(y: torch.Tensor, cos: torch.Tensor, hq: int, hkv: int) -> bool:
    W = y.shape[-1]
    if y.dim() != 3 or W % (hq + 2 * hkv):
        return False
    D = W // (hq + 2 * hkv)
    return (_FUSED_ATTN and _FUSED_ACT and D in (64, 128) and y.is_cuda and y.dtype == torch.bfloat16
            and y.is_contiguous() and y.data_ptr() % 16 == 0 and cos.dtype == torch.float32 and cos.is_cuda
            and cos.dim() == 2 and cos.shape[0] >= y.shape[1] and cos.shape[1] * 2 == D and hq % hkv == 0)


def rope_attention_packed(y: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, hq: int, hkv: int,
                          causal: bool = True, scale: Optional[float] = None) -> torch.Tensor:
    """Rotary embedding + (causal, grouped-query) attention of a packed q | k | v projection
    y [B, S, (hq + 2 hkv) * D]; returns [B, S, hq, D].  Callers check rope_attention_packed_ok."""
    D = y.shape[-1] // (hq + 2 * hkv)
    sc = float(scale) if scale is not None else 1.0 / (D ** 0.5)
    return _RopeAttentionPacked.apply(y, cos, sin, int(hq), int(hkv), bool(causal), sc)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False,
              scale: Optional[float] = None, kv_len: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Scaled dot-product attention on the [batch, seq, heads, head_dim] layout (the projection
    outputs viewed per head, no transposes): q [B, Sq, Hq, D], k / v [B, Sk, Hkv, D] with Hq a
    multiple of Hkv (grouped-query attention), optional causal mask (Sq == Sk) and key padding
    (``kv_len`` int32 [B]: keys >= kv_len[b] are masked).  Returns [B, Sq, Hq, D].

    bf16 device operands with head dim 64 / 128 run the hipps flash-attention kernels; anything
    else runs ``F.scaled_dot_product_attention`` on the transposed views."""
    D = q.shape[-1]
    sc = float(scale) if scale is not None else 1.0 / (D ** 0.5)
    if attention_ok(q, k, v, causal):
        kl = None
        if kv_len is not None:
            kl = kv_len.to(device=q.device, dtype=torch.int32).contiguous()
        return _FlashAttention.apply(q, k, v, bool(causal), sc, kl)
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    if k.shape[2] != q.shape[2]:
        rep = q.shape[2] // k.shape[2]
        kt, vt = kt.repeat_interleave(rep, dim=1), vt.repeat_interleave(rep, dim=1)
    mask = None
    if kv_len is not None:
        keys = torch.arange(k.shape[1], device=q.device)
        mask = (keys[None, :] < kv_len.to(q.device).view(-1, 1))[:, None, None, :]
        if causal:
            mask = mask & torch.ones(q.shape[1], k.shape[1], dtype=torch.bool, device=q.device).tril()
            causal = False
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask, is_causal=causal, scale=sc)
    return o.transpose(1, 2)


def _flat16_ok(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
               and t.data_ptr() % 16 == 0 for t in ts)


class _SwiGLU(torch.autograd.Function):
    """silu(a) * b on bf16 (csrc/act.hip): one pass forward (read a, b; write c), one pass
    backward (read g, a, b; write da, db) instead of 2 + 4 eager kernels."""

    @staticmethod
    def forward(ctx, a, b):
        c = torch.empty_like(a)
        native().swiglu_forward(a, b, c)
        ctx.save_for_backward(a, b)
        return c

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.to(torch.bfloat16).contiguous()
        da, db = torch.empty_like(a), torch.empty_like(b)
        native().swiglu_backward(g, a, b, da, db)
        return da, db


class _SwiGLUPacked(torch.autograd.Function):
    """silu(y[:, :F]) * y[:, F:] of ONE packed gate / up projection y [.., 2F] (csrc/act.hip
    k_swiglu_*_rows): the backward writes the packed [.., 2F] gradient directly."""

    @staticmethod
    def forward(ctx, y):
        F2 = y.shape[-1]
        y2 = y.reshape(-1, F2)
        c = torch.empty(y2.shape[0], F2 // 2, dtype=y.dtype, device=y.device)
        native().swiglu_rows_forward(y2, c)
        ctx.save_for_backward(y)
        return c.view(*y.shape[:-1], F2 // 2)

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        F2 = y.shape[-1]
        g2 = g.to(torch.bfloat16).reshape(-1, F2 // 2)
        if g2.stride(-1) != 1 or g2.stride(0) % 8 or g2.data_ptr() % 16:
            g2 = g2.contiguous()
        dy = torch.empty_like(y)
        native().swiglu_rows_backward(g2, y.reshape(-1, F2), dy.view(-1, F2))
        return dy


def swiglu_packed(y: torch.Tensor) -> torch.Tensor:
    """F.silu(a) * b for a, b = the two halves of y's last dimension (a fused gate / up GEMM)."""
    F2 = y.shape[-1]
    if (_FUSED_ACT and y.is_cuda and y.dtype == torch.bfloat16 and y.is_contiguous() and F2 % 16 == 0
            and y.data_ptr() % 16 == 0):
        return _SwiGLUPacked.apply(y)
    a, b = y.split(F2 // 2, dim=-1)
    return F.silu(a) * b


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """F.silu(a) * b (the Llama MLP gate) on the fused kernel for bf16 device tensors."""
    if _FUSED_ACT and a.shape == b.shape and _flat16_ok(a, b):
        return _SwiGLU.apply(a, b)
    return F.silu(a) * b


class _LayerNorm(torch.autograd.Function):
    """LayerNorm over the last dim of a bf16 activation with fp32 weight / bias (csrc/ln.hip): no
    per-forward casts of the parameters, fp32 weight / bias gradients written directly."""

    @staticmethod
    def forward(ctx, x, w, b, eps, colsum_dx=False):
        D = x.shape[-1]
        y = torch.empty_like(x)
        R = x.numel() // D
        mean = torch.empty(R, dtype=torch.float32, device=x.device)
        rstd = torch.empty(R, dtype=torch.float32, device=x.device)
        native().ln_forward(x, w, b, y, mean, rstd, float(eps))
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.colsum_dx = bool(colsum_dx)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x)
        dw, db = torch.empty_like(w), torch.empty_like(w)
        cs = torch.empty_like(w) if ctx.colsum_dx else None
        native().ln_backward(dy, x, mean, rstd, w, dx, dw, db, cs)
        if cs is not None:
            stash_colsum(dx, cs)
        return dx, dw, db, None, None


def layer_norm_ok(x: torch.Tensor, weight, bias) -> bool:
    """Can _LayerNorm run F.layer_norm(x, (D,), weight, bias) (bf16 x, fp32 affine params)?"""
    D = x.shape[-1] if x.dim() else 0
    return (_FUSED_ACT and weight is not None and bias is not None and x.is_cuda and x.dtype == torch.bfloat16
            and x.is_contiguous() and D % 8 == 0 and 8 <= D <= 2048 and x.data_ptr() % 16 == 0
            and all(p.dtype == torch.float32 and p.is_contiguous() and p.numel() == D and p.data_ptr() % 16 == 0
                    for p in (weight, bias)))


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float,
               colsum_dx: bool = False) -> torch.Tensor:
    """F.layer_norm over the last dim on the fused kernels (callers check layer_norm_ok).
    ``colsum_dx``: x is a biased Linear's output -- the backward also sums dx over the rows and
    leaves it for that Linear's bias gradient (stash_colsum / colsum_f32)."""
    return _LayerNorm.apply(x, weight, bias, eps, colsum_dx)


class _RMSNorm(torch.autograd.Function):
    """RMSNorm over the last dim (csrc/ln.hip): reads the fp32 residual stream (or bf16) directly
    -- no cast kernel -- writes bf16; the backward writes dx in x's dtype (the fp32 residual
    gradient, no cast back) and the fp32 weight gradient."""

    @staticmethod
    def forward(ctx, x, w, eps):
        D = x.shape[-1]
        y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        rstd = torch.empty(x.numel() // D, dtype=torch.float32, device=x.device)
        native().rms_forward(x, w, y, rstd, float(eps))
        ctx.save_for_backward(x, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        native().rms_backward(dy, x, rstd, w, dx, dw)
        return dx, dw, None


def rms_norm_ok(x: torch.Tensor, weight) -> bool:
    """Can _RMSNorm run (fp32 / bf16 contiguous x, D % 8 == 0, D <= 4096, fp32 weight)?"""
    D = x.shape[-1] if x.dim() else 0
    return (_FUSED_ACT and weight is not None and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)
            and x.is_contiguous() and D % 8 == 0 and 8 <= D <= 4096 and x.data_ptr() % 16 == 0
            and weight.dtype == torch.float32 and weight.is_contiguous() and weight.numel() == D
            and weight.data_ptr() % 16 == 0)


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """bf16 RMSNorm of x over the last dim on the fused kernels (callers check rms_norm_ok)."""
    return _RMSNorm.apply(x, weight, eps)


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


class _AddRMSNorm(torch.autograd.Function):
    """Residual add + RMSNorm in one pass (csrc/ln.hip k_rms_fwd with ``addy``): s = x + y (x the
    fp32 residual stream, y a block's bf16 output) is written once and normalised from registers
    -- no separate add kernel that writes s and a norm that reads it back.  The backward folds the
    residual stream's own gradient into the norm's dx (k_rms_bwd with ``dres``) and emits its bf16
    twin for y: one pass instead of norm backward + autograd's fp32 add + a bf16 cast."""

    @staticmethod
    def forward(ctx, x, y, w, eps):
        D = x.shape[-1]
        s = torch.empty_like(x)
        h = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        rstd = torch.empty(x.numel() // D, dtype=torch.float32, device=x.device)
        native().rms_forward(x, w, h, rstd, float(eps), y, s)
        ctx.save_for_backward(s, w, rstd)
        ctx.set_materialize_grads(False)
        return s, h

    @staticmethod
    def backward(ctx, ds, dh):
        s, w, rstd = ctx.saved_tensors
        dh = torch.zeros(s.shape, dtype=torch.bfloat16, device=s.device) if dh is None else \
            _aligned(dh.to(torch.bfloat16))
        dres = None if ds is None else _aligned(ds.to(torch.float32))
        dx = torch.empty_like(s)
        dy = torch.empty(s.shape, dtype=torch.bfloat16, device=s.device) if ctx.needs_input_grad[1] else None
        dw = torch.empty_like(w)
        native().rms_backward(dh, s, rstd, w, dx, dw, dres, dy)
        return dx, dy, dw, None


def add_rms_norm_ok(x: torch.Tensor, y: torch.Tensor, weight) -> bool:
    """Can _AddRMSNorm run: fp32 residual x and bf16 y of x's shape, both contiguous and aligned?"""
    return (rms_norm_ok(x, weight) and x.dtype == torch.float32 and y.dtype == torch.bfloat16
            and y.shape == x.shape and y.is_contiguous() and y.data_ptr() % 16 == 0 and y.device == x.device)


def add_rms_norm(x: torch.Tensor, y: torch.Tensor, weight: torch.Tensor, eps: float):
    """(x + y, bf16 RMSNorm(x + y)) in one fused pass each way (callers check add_rms_norm_ok)."""
    return _AddRMSNorm.apply(x, y, weight, eps)


class _Embed3(torch.autograd.Function):
    """bf16 word + position + token-type embedding of ids [B, S] (csrc/embed.hip): one gather-add
    pass forward; backward the position gradient as a fixed-order batch sum, the word (and
    explicit type) gradient by one wave per id over the stably sorted rows, the all-zero type ids'
    gradient as a column sum -- deterministic, in place of PyTorch's embedding_dense_backward
    chains (~1 ms per BERT-base step at batch 32)."""

    @staticmethod
    def forward(ctx, ids, word, pos, typ, tt):
        B, S = ids.shape
        out = torch.empty((B, S, word.shape[1]), dtype=torch.bfloat16, device=ids.device)
        native().embed_forward(ids, tt, word, pos, typ, out)
        ctx.save_for_backward(ids, tt)
        ctx.shapes = (word.shape, pos.shape, typ.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, tt = ctx.saved_tensors
        (V, D), (P, _), (T, _) = ctx.shapes
        B, S = ids.shape
        d2 = _aligned(dout.to(torch.bfloat16)).view(-1, D)
        C = native()
        dword = dpos = dtyp = None

        def seg(keys, rows):
            g = torch.zeros((rows, D), dtype=torch.float32, device=d2.device)
            sid, perm = torch.sort(keys.reshape(-1), stable=True)
            C.embed_seg_backward(d2, sid, perm, g)
            return g

        if ctx.needs_input_grad[1]:
            dword = seg(ids, V)
        if ctx.needs_input_grad[2]:
            dpos = torch.empty((P, D), dtype=torch.float32, device=d2.device)
            C.embed_pos_backward(d2, dpos, B, S)
        if ctx.needs_input_grad[3]:
            if tt is None:
                dtyp = torch.zeros((T, D), dtype=torch.float32, device=d2.device)
                dtyp[0] = colsum_f32(d2)
            else:
                dtyp = seg(tt, T)
        return None, dword, dpos, dtyp, None


_FUSED_EMBED = _os.environ.get("HIPPS_FUSED_EMBED", "1") != "0"


def bert_embed_ok(ids: torch.Tensor, word, pos, typ) -> bool:
    """Can _Embed3 run: bf16 autocast, int64 [B, S] device ids, fp32 contiguous aligned tables with
    D % 8 == 0 and S within the position table?"""
    D = word.shape[-1]
    return (_FUSED_EMBED and ids.is_cuda and ids.dtype == torch.int64 and ids.dim() == 2
            and torch.is_autocast_enabled() and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and D % 8 == 0 and ids.shape[1] <= pos.shape[0]
            and all(t.dtype == torch.float32 and t.is_contiguous() and t.dim() == 2 and t.shape[1] == D
                    and t.data_ptr() % 16 == 0 and t.is_cuda for t in (word, pos, typ)))


def bert_embed(ids: torch.Tensor, word: torch.Tensor, pos: torch.Tensor, typ: torch.Tensor, type_ids=None):
    """bf16 word[ids] + pos[:S] + typ[type_ids or 0] (callers check bert_embed_ok)."""
    if type_ids is not None:
        type_ids = type_ids.to(torch.int64).contiguous()
    return _Embed3.apply(ids.contiguous(), word, pos, typ, type_ids)


class _Rope(torch.autograd.Function):
    """Rotary embedding of interleaved pairs on x [B, S, H, hd] bf16 (csrc/act.hip k_rope, fp32
    cos / sin tables [S, hd/2]); the backward is the rotation by -theta."""

    @staticmethod
    def forward(ctx, x, cos, sin):
        B, S, H, hd = x.shape
        y = torch.empty_like(x)
        native().rope_apply(x.view(B * S, H * hd), y.view(B * S, H * hd), cos, sin, S, hd, 1.0)
        ctx.save_for_backward(cos, sin)
        return y

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        B, S, H, hd = g.shape
        g = g.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(g)
        native().rope_apply(g.view(B * S, H * hd), dx.view(B * S, H * hd), cos, sin, S, hd, -1.0)
        return dx, None, None


def rope_ok(x: torch.Tensor, cos: torch.Tensor) -> bool:
    """Can _Rope rotate x [B, S, H, hd] with fp32 tables cos [S, hd/2]?"""
    return (_FUSED_ACT and x.dim() == 4 and x.shape[-1] % 8 == 0 and _flat16_ok(x) and cos.dtype == torch.float32
            and cos.is_cuda and cos.dim() == 2 and cos.shape[0] >= x.shape[1] and cos.shape[1] * 2 == x.shape[-1])


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x rotated pairwise (x[2i], x[2i+1]) by angle pos * theta_i (cos / sin: fp32 [S, hd/2]) on the
    fused kernel; callers check rope_ok first."""
    return _Rope.apply(x, cos, sin)


class _Conv1x1(torch.autograd.Function):
    """1x1 convolution on channels-last bf16 as an MFMA GEMM (hipps/csrc/gemm.hip) that also
    emits the per-channel batch statistics of its output for the BatchNorm that follows.
    Backward: the input gradient of a stride-1 conv is the same NT GEMM against the transposed
    weight (dX[M,Cin] = dY[M,Cout] . W[Cout,Cin]); the weight gradient is the split-M MFMA
    reduction with transposing LDS reads (conv1x1_wgrad), written straight into an fp32 grad
    for an fp32 master weight (no bf16 round trip); strided dgrad goes to MIOpen.
    Other gradient paths into x are summed in the dgrad epilogue: a ResidualTap's (dy * bits),
    and with ``alias`` the gradient of the returned alias of x (e.g. a downsample branch)."""

    @staticmethod
    def forward(ctx, x, w_master, stride, tap=None, alias=False, bngrad=None, s2tap=None):
        w = bf16_weight(w_master)
        ctx.wdtype = w_master.dtype
        ctx.wparam = w_master
        # no zero-filled grad for the non-differentiable BN partials (a 12.8 MB fill per layer)
        ctx.set_materialize_grads(False)
        ctx.wt = _TSHADOWS.get(w_master.data_ptr()) if w_master.dtype == torch.float32 else None
        ctx.bngrad = bngrad if stride == 1 else None
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        part = _conv1x1_gemm(x, w.reshape(Cout, Cin), y, H, W, stride, True)
        ctx.stride = stride
        ctx.tap = tap
        # alias (conv1): the downsample's compact gradient arrives here; stride 2 (downsample): put
        # it here
        ctx.s2tap = s2tap if (_S2TAP and ((alias and stride == 1) or stride == 2)) else None
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        if alias:
            return y, part, x  # an input returned as-is becomes a view whose grad comes back here
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart, d_alias=None):
        x, w = ctx.saved_tensors
        s = ctx.stride
        s2tap, ctx.s2tap = ctx.s2tap, None
        if dy is None:  # y unused (grads are not materialized): only the alias path carries a grad
            ctx.bngrad = None
            if s2tap is not None and s2tap.dx is not None:
                raise RuntimeError("compact stride-2 gradient without a consuming dgrad")
            return d_alias, None, None, None, None, None, None
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        add, add_mask = ctx.tap.take() if ctx.tap is not None else (None, None)
        add_s2 = False
        if s2tap is not None and s == 1 and s2tap.dx is not None:  # conv1: the downsample's gradient
            if d_alias is not None or add is not None:
                raise RuntimeError("compact stride-2 gradient next to another alias / tap gradient")
            add, add_s2 = s2tap.dx, True
            s2tap.dx = None
        if d_alias is not None:
            d_alias = d_alias.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            if add is None:
                add = d_alias
            else:  # both paths present (not produced by the ResNet blocks): fold eagerly
                add = _masked(add, add_mask, x.shape[1]) + d_alias
                add_mask = None
        own_dx = ctx.needs_input_grad[0] and s == 1
        s2_dx = (ctx.needs_input_grad[0] and s == 2 and s2tap is not None and x.shape[1] % 64 == 0 and
                 dy.shape[1] % 64 == 0)
        if ctx.needs_input_grad[0] and not own_dx and not s2_dx:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
            if add is not None:
                dx = dx + _masked(add, add_mask, x.shape[1])
        if ctx.needs_input_grad[1] and not _OWN_WGRAD:
            dw = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1].to(ctx.wdtype)
        elif ctx.needs_input_grad[1]:
            def wg():
                d = torch.empty(w.shape, dtype=torch.float32, device=w.device)
                _conv_wgrad(dy, x, d, 1, 1, s, 0)
                return d if ctx.wdtype == torch.float32 else d.to(ctx.wdtype)

            dw = _on_wgrad_stream(ctx.wparam, (dy, x), wg)
        ctx.wparam = None
        if s2_dx:  # compact gradient at the output positions, summed in conv1's dgrad epilogue
            cout, cin = w.shape[0], w.shape[1]
            wt = ctx.wt if ctx.wt is not None else w.reshape(cout, cin).t().contiguous()
            n, _, ho, wo = dy.shape
            dxc = torch.empty((n, cin, ho, wo), dtype=torch.bfloat16, device=dy.device,
                              memory_format=torch.channels_last)
            _conv1x1_gemm(dy, wt, dxc, ho, wo, 1, False)
            s2tap.dx = dxc
            dx = None
        if own_dx:
            cout, cin = w.shape[0], w.shape[1]
            wt = ctx.wt  # [Cin, Cout]: K-contiguous B operand (refreshed with the weight shadow)
            if wt is None:
                wt = w.reshape(cout, cin).t().contiguous()
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            bg = ctx.bngrad
            # x's gradient is complete here only if the residual path it also feeds was summed in
            # (an identity block's tap delivered, or no tap was involved)
            if bg is not None and (ctx.tap is None or add is not None):
                bg.part = _conv1x1_gemm(dy, wt, dx, x.shape[2], x.shape[3], 1, True, add, add_mask, bg, add_s2)
            else:
                _conv1x1_gemm(dy, wt, dx, x.shape[2], x.shape[3], 1, False, add, add_mask, None, add_s2)
        ctx.bngrad = None
        return dx, dw, None, None, None, None, None


class _BNReluConv1x1(torch.autograd.Function):
    """conv1x1(relu(bn(x))) for a training-mode BatchNorm whose output only feeds this stride-1
    1x1 conv (ResNet bn2 -> conv3): the BN's statistics (reduce + finalize, no apply pass), then
    the MFMA GEMM reading relu(x * scale + shift) in its operand prologue (gemm.hip bn_relu8; the
    same bf16 rounding as the apply kernel), with the next BN's statistics in its epilogue.  The
    BN output is never written or re-read.  Backward: the input-gradient GEMM with this BN's
    backward reduction in its epilogue (relu' recomputed from x), the BN backward apply, and the
    weight gradient with the same prologue on its X operand."""

    @staticmethod
    def forward(ctx, x, bn_w, bn_b, running_mean, running_var, eps, momentum, w_master):
        w = bf16_weight(w_master)
        ctx.wdtype = w_master.dtype
        ctx.set_materialize_grads(False)
        ctx.wt = _TSHADOWS.get(w_master.data_ptr()) if w_master.dtype == torch.float32 else None
        n, c, h, wd = x.shape
        cout = w.shape[0]
        f32 = dict(dtype=torch.float32, device=x.device)
        mean, invstd, scale, shift = (torch.empty(c, **f32) for _ in range(4))
        native().bn_forward_stats(x, bn_w, bn_b, running_mean, running_var, mean, invstd, scale, shift, c, float(eps),
                                  float(momentum))
        y = torch.empty((n, cout, h, wd), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        part = torch.empty((2, cout, native().conv1x1_mtiles(n * h * wd)), **f32)
        native().conv1x1_forward(x, w.reshape(cout, c), y, part, h, wd, 1, pro_scale=scale, pro_shift=shift)
        ctx.save_for_backward(x, w, bn_w, mean, invstd, scale, shift)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w, bn_w, mean, invstd, scale, shift = ctx.saved_tensors
        if dy is None:
            return (None,) * 8
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, c, h, wd = x.shape
        cout = w.shape[0]
        wt = ctx.wt if ctx.wt is not None else w.reshape(cout, c).t().contiguous()
        # gradient of the (never materialised) BN output + that BN's backward reduction
        dbn = torch.empty_like(x, memory_format=torch.channels_last)
        part = torch.empty((2, c, native().conv1x1_mtiles(n * h * wd)), dtype=torch.float32, device=x.device)
        native().conv1x1_forward(dy, wt, dbn, part, h, wd, 1, None, None, x, None, mean, invstd, scale, shift)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dgw, dgb = torch.empty_like(bn_w), torch.empty_like(bn_w)
        native().bn_backward_partials(part, part.shape[2], dbn, x, MASK_X, bn_w, mean, invstd, scale, shift, dx, None,
                                      dgw, dgb, c, None)
        dw = None
        if ctx.needs_input_grad[7]:
            dw = torch.empty(w.shape, dtype=torch.float32, device=w.device)
            native().conv1x1_wgrad(dy, x, dw.view(cout, c), h, wd, 1, scale, shift)
            if ctx.wdtype != torch.float32:
                dw = dw.to(ctx.wdtype)
        return dx, dgw, dgb, None, None, None, None, dw


def bn_relu_conv1x1_ok(bn, conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Can _BNReluConv1x1 run conv(relu(bn(x)))?"""
    return (bn.training and getattr(bn, "relu", False) and bn._fast_ok(x, None) and conv.stride == (1, 1)
            and conv1x1_ok(conv, x) and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def bn_relu_conv_bn(bn, conv: nn.Conv2d, bn_next, x, residual=None, res_tap=None):
    """bn_next(conv(relu(bn(x))), residual) with bn's apply folded into the conv's operand prologue
    (_BNReluConv1x1); callers check bn_relu_conv1x1_ok first."""
    bn._nbt_pending += 1
    y, part = _BNReluConv1x1.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum,
                                   conv.weight)
    if bn_next._fast_ok(y, residual):
        return bn_next(y, residual, stats=part, res_tap=res_tap)
    return bn_next(y, residual)


class _ConvKxK(torch.autograd.Function):
    """KxK convolution on channels-last bf16: forward and input gradient on MIOpen, weight
    gradient on the hipps implicit-GEMM MFMA kernel (conv_wgrad), written straight into an fp32
    gradient for the fp32 master weight.  MIOpen's 3x3 weight-gradient kernels accumulate in an
    fp32 workspace and need 3 extra zero-fill / cast kernels per call (profiles/bench_n1_steady_r1d.txt)."""

    @staticmethod
    def forward(ctx, x, w_master, stride, pad, own_wgrad=True, stats=False, bngrad=None):
        w = bf16_weight(w_master)
        ctx.wdtype = w_master.dtype
        ctx.wparam = w_master
        ctx.own_wgrad = own_wgrad
        # x is the output of a fused BN whose only gradient is this conv's input gradient: the
        # input gradient (stride 1: a forward conv on gemm2; stride 2: the parity GEMMs) reduces
        # that BN's backward statistics in its epilogue
        ctx.bngrad = bngrad if stride == 1 else None
        ctx.bngrad_s2 = bngrad if stride == 2 else None
        ctx.set_materialize_grads(False)
        ctx.wf = _TSHADOWS.get(w_master.data_ptr()) if w_master.dtype == torch.float32 else None
        part = None
        if _GEMM2 and w.is_contiguous(memory_format=torch.channels_last):
            y, part = _convkxk_gemm(x, w, stride, pad, stats)  # the next BN's statistics from the epilogue
        elif _own_kxk(x.shape[1], w.shape[0]):
            n, _, h, wd = x.shape
            k = w.shape[2]
            ho, wo = (h + 2 * pad - k) // stride + 1, (wd + 2 * pad - k) // stride + 1
            y = torch.empty((n, w.shape[0], ho, wo), dtype=torch.bfloat16, device=x.device,
                            memory_format=torch.channels_last)
            if stats:  # the following BatchNorm's statistics from the GEMM epilogue
                part = torch.empty((2, w.shape[0], native().conv1x1_mtiles(n * ho * wo)), dtype=torch.float32,
                                   device=x.device)
            native().convkxk_forward(x, w, y, part, stride, pad)
        else:
            y = torch.ops.aten.convolution(x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)
        ctx.geom = (stride, pad)
        ctx.save_for_backward(x, w)
        if part is None:
            part = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        x, w = ctx.saved_tensors
        s, p = ctx.geom
        bg, ctx.bngrad = ctx.bngrad, None
        if dy is None:
            ctx.bngrad_s2 = None
            return None, None, None, None, None, None, None
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        k = w.shape[2]
        if ctx.needs_input_grad[0] and _DGRAD_AS_FWD and s == 1 and k == w.shape[3] and 2 * p == k - 1:
            # dx[n, ci] = sum_co conv(dy[n, co], rot180(W[co, ci])) with the same padding
            wf = ctx.wf if ctx.wf is not None and ctx.wf.dim() == 4 else None
            if wf is None:
                wf = torch.flip(w, (2, 3)).transpose(0, 1).contiguous(memory_format=torch.channels_last)
            if _GEMM2 and wf.is_contiguous(memory_format=torch.channels_last):
                dx, part = _convkxk_gemm(dy, wf, 1, p, False, bg)
                if bg is not None:
                    bg.part = part  # None when MIOpen ran: the BN backward then reduces itself
            elif _own_kxk(dy.shape[1], wf.shape[0]):
                dx = torch.empty_like(x, memory_format=torch.channels_last)
                native().convkxk_forward(dy, wf, dx, None, 1, p)
            else:
                dx = torch.ops.aten.convolution(dy, wf, None, [1, 1], [p, p], [1, 1], False, [0, 0], 1)
        elif (ctx.needs_input_grad[0] and _DGRAD_S2 and s == 2 and p == 1 and k == 3 and w.shape[3] == 3 and
              x.shape[1] % 64 == 0 and dy.shape[1] % 64 == 0):
            # stride-2 3x3: four output-parity GEMMs (no zero fill), bn1's reduction in the epilogue
            wf = ctx.wf if ctx.wf is not None and ctx.wf.dim() == 4 else None
            if wf is None:
                wf = torch.flip(w, (2, 3)).transpose(0, 1).contiguous(memory_format=torch.channels_last)
            bg2 = getattr(ctx, "bngrad_s2", None)
            ctx.bngrad_s2 = None
            dx, part = _dgrad_s2(dy, x, w, wf, bg2)
            if bg2 is not None:
                bg2.part = part
        elif ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        if ctx.needs_input_grad[1] and not ctx.own_wgrad:
            dw = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1].to(ctx.wdtype)
        elif ctx.needs_input_grad[1]:
            def wg():
                d = torch.empty(w.shape, dtype=torch.float32, device=w.device, memory_format=torch.channels_last)
                _conv_wgrad(dy, x, d, w.shape[2], w.shape[3], s, p)
                return d if ctx.wdtype == torch.float32 else d.to(ctx.wdtype)

            dw = _on_wgrad_stream(ctx.wparam, (dy, x), wg)
        ctx.wparam = None
        return dx, dw, None, None, None, None, None


def _own_kxk(cin: int, cout: int) -> bool:
    """Route this KxK forward to hipps' implicit-GEMM kernel (gemm.hip convkxk_forward)?"""
    return _OWN_KXK_FWD and cin % 64 == 0 and cout % 64 == 0


def convkxk_ok(conv: nn.Conv2d, x: torch.Tensor, own_wgrad: bool = True) -> bool:
    """Can _ConvKxK run this (square, zero-padded, dense) convolution (with the hipps weight
    gradient when ``own_wgrad``)?"""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and torch.is_grad_enabled() and
            x.is_contiguous(memory_format=torch.channels_last)):
        return False
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if k[0] != k[1] or s[0] != s[1] or not isinstance(p, tuple) or p[0] != p[1] or conv.dilation != (1, 1):
        return False
    if conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    w = conv.weight
    if not own_wgrad:
        return w.is_contiguous(memory_format=torch.channels_last)
    # 64-channel KxK layers: the first core's 64x64 output tile re-reads both operands once per tap
    # and MIOpen is faster there (0.23 vs 0.29 ms at 64x56x56, profiles/conv3x3_wgrad.json); with
    # gemm2 the tuner measures its 128x128-tile kernel against MIOpen for them
    cmin = 64 if _GEMM2 else 128
    return (conv.in_channels % cmin == 0 and conv.out_channels % 64 == 0 and
            w.is_contiguous(memory_format=torch.channels_last))


class _StemConv(torch.autograd.Function):
    """ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels) on the hipps MFMA kernels
    (csrc/stem.hip): forward with the following BatchNorm's partial statistics in the epilogue,
    fp32 weight gradient straight into the master's dtype; an input gradient (never needed for an
    image batch) falls back to MIOpen."""

    @staticmethod
    def forward(ctx, x, w_master, stats=True):
        w = bf16_weight(w_master).contiguous(memory_format=torch.channels_last)
        n, _, h, wd = x.shape
        ho, wo = (h - 1) // 2 + 1, (wd - 1) // 2 + 1
        y = torch.empty((n, 64, ho, wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        part = (torch.empty((2, 64, native().stem_mtiles(n, ho)), dtype=torch.float32, device=x.device) if stats
                else torch.empty(0, device=x.device))
        native().stem_forward(x, w, y, part if stats else None)
        ctx.wdtype = w_master.dtype
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        x, w = ctx.saved_tensors
        if dy is None:
            return None, None, None
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            dw = torch.empty((64, 3, 7, 7), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
            native().stem_wgrad(dy, x, dw)
            if ctx.wdtype != torch.float32:
                dw = dw.to(ctx.wdtype)
        return dx, dw, None


def stem_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Can _StemConv run this convolution on this input (after the autocast cast)?"""
    if not (_OWN_STEM and x.is_cuda and x.dim() == 4 and x.shape[1] == 3):
        return False
    if x.dtype != torch.bfloat16 and not (x.dtype == torch.float32 and torch.is_autocast_enabled("cuda") and
                                          torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    if (conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding, conv.dilation,
            conv.groups) != (3, 64, (7, 7), (2, 2), (3, 3), (1, 1), 1):
        return False
    if conv.bias is not None or conv.padding_mode != "zeros":
        return False
    h, w = x.shape[2], x.shape[3]
    return w % 8 == 0 and h >= 7 and w >= 7 and (w - 1) // 2 + 1 <= 128


def conv2d_stats(conv: nn.Conv2d, x: torch.Tensor, fuse: bool = True, bn_grad: bool = False):
    """(conv(x), part): with the hipps implicit-GEMM forward, ``part`` holds the following
    BatchNorm's partial statistics [2, Cout, m_tiles] from its epilogue (None otherwise); the
    hipps weight gradient when eligible (see _ConvKxK).  ``bn_grad``: x is the output of a fused
    BN whose only consumer is this conv (see BNGradTap)."""
    if fuse and stem_ok(conv, x):
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y, part = _StemConv.apply(xb, conv.weight, conv.training)
        return y, (part if part.numel() else None)
    bg = getattr(x, "_hipps_bngrad", None) if bn_grad else None
    if fuse and conv.training and convkxk_ok(conv, x):
        y, part = _ConvKxK.apply(x, conv.weight, conv.stride[0], conv.padding[0], True, True, bg)
        return y, (part if part.numel() else None)
    if conv.training and convkxk_ok(conv, x, own_wgrad=False) and (
            (_DGRAD_AS_FWD and conv.stride[0] == 1) or _own_kxk(conv.in_channels, conv.out_channels) or _GEMM2):
        y, part = _ConvKxK.apply(x, conv.weight, conv.stride[0], conv.padding[0], False, True, bg)  # MIOpen wgrad
        return y, (part if part.numel() else None)
    return conv(x), None


def conv2d(conv: nn.Conv2d, x: torch.Tensor, fuse: bool = True) -> torch.Tensor:
    """conv(x) with the hipps kernels when eligible (see _ConvKxK); otherwise conv(x)."""
    return conv2d_stats(conv, x, fuse)[0]


def conv2d_bn(conv: nn.Conv2d, bn, x: torch.Tensor, residual=None, fuse: bool = True, bn_grad: bool = False):
    """bn(conv(x), residual) with the BN statistics from the conv's GEMM epilogue when available
    (``bn_grad``: see conv2d_stats)."""
    y, part = conv2d_stats(conv, x, fuse, bn_grad)
    if part is not None and bn.training and bn._fast_ok(y, residual):
        return bn(y, residual, stats=part)
    return bn(y, residual)


def _masked(t, mask, C):
    """t * ReLU bits (uint8, bit j of byte i = element 8i+j of the channels-last storage)."""
    if mask is None:
        return t
    bits = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    flat = t.permute(0, 2, 3, 1).reshape(-1) * bits.view(-1).to(t.dtype)
    return flat.view(t.shape[0], t.shape[2], t.shape[3], C).permute(0, 3, 1, 2)


def conv1x1_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Can the MFMA 1x1 path run this convolution on this input?"""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and
            x.is_contiguous(memory_format=torch.channels_last)):
        return False
    if conv.kernel_size != (1, 1) or conv.padding != (0, 0) or conv.dilation != (1, 1) or conv.groups != 1:
        return False
    if conv.bias is not None or conv.stride[0] != conv.stride[1]:
        return False
    return conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0


def conv1x1_stats(x, weight, stride=1, tap=None, alias=False, bngrad=None, s2tap=None):
    """(y, part[, x_alias]): bf16 1x1 conv output and its [2, Cout, m_tiles] BN partial
    statistics (see _Conv1x1 for ``tap`` / ``alias``, BNGradTap for ``bngrad``, S2Tap for
    ``s2tap``)."""
    return _Conv1x1.apply(x, weight, int(stride), tap, bool(alias), bngrad, s2tap)


class _FusedBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, eps, momentum, relu, part=None, tap=None):
        C = x.shape[1]
        y = torch.empty_like(x, memory_format=torch.channels_last)
        f32 = dict(dtype=torch.float32, device=x.device)
        mean, invstd = torch.empty(C, **f32), torch.empty(C, **f32)
        scale, shift = torch.empty(C, **f32), torch.empty(C, **f32)
        # relu(bn(x) + res): the mask depends on res, so keep 1 bit per element instead of
        # re-reading the bf16 output in the backward
        mode = MASK_NONE if not relu else (MASK_BITS if res is not None else MASK_X)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) if mode == MASK_BITS else None
        if part is not None:  # statistics already reduced by the producing 1x1 conv
            native().bn_forward_partials(part, part.shape[2], x, res, y, weight, bias, running_mean, running_var,
                                         mean, invstd, scale, shift, C, float(eps), float(momentum), bool(relu), mask)
        else:
            native().bn_forward_train(x, res, y, weight, bias, running_mean, running_var, mean, invstd, scale, shift,
                                      C, float(eps), float(momentum), bool(relu), mask)
        ctx.mode, ctx.C, ctx.has_res = mode, C, res is not None
        # the residual gradient is dy * bits (or dy): hand it to the consumer through the tap
        ctx.tap = tap if (res is not None and mode in (MASK_NONE, MASK_BITS)) else None
        ctx.save_for_backward(x, mask, weight, mean, invstd, scale, shift)
        # a consuming 1x1 conv may reduce this BN's backward statistics for it (BNGradTap)
        ctx.bngrad = None
        if mode in (MASK_X, MASK_BITS):
            ctx.bngrad = BNGradTap(x, mask, mean, invstd, scale, shift)
            y._hipps_bngrad = ctx.bngrad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd, scale, shift = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        tap = ctx.tap
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res and tap is None else None
        dw = torch.empty_like(weight)
        db = torch.empty_like(weight)
        bg, ctx.bngrad = ctx.bngrad, None
        if bg is not None and bg.part is not None:  # reduction already done in the consumer's epilogue
            native().bn_backward_partials(bg.part, bg.part.shape[2], dy, x, ctx.mode, weight, mean, invstd, scale,
                                          shift, dx, dres, dw, db, ctx.C, mask)
            bg.part = None
        else:
            native().bn_backward(dy, x, None, ctx.mode, weight, mean, invstd, scale, shift, dx, dres, dw, db, ctx.C,
                                 mask)
        if tap is not None:
            tap.dy, tap.mask = dy, (mask if ctx.mode == MASK_BITS else None)
        return dx, dres, dw, db, None, None, None, None, None, None, None


class _DualBNRelu(torch.autograd.Function):
    """z = relu(bn3(x3) + bnd(xd)) for a ResNet downsample block, both training BNs' statistics
    from their convs' epilogues: the downsample BN is applied inside bn3's apply pass
    (norm.hip bn_dual_forward), so its output -- the residual -- is never written or re-read.
    Backward (bn_dual_backward): bn3's input gradient and the downsample BN's reduction in one
    pass (the residual gradient dz * bits is recomputed, never stored), then the downsample BN's
    input gradient.  bn3's backward reduction may come from the consumer's dgrad epilogue
    (BNGradTap on z, as for _FusedBNAct)."""

    @staticmethod
    def forward(ctx, x3, part3, w3, b3, rm3, rv3, eps3, mom3, xd, partd, wd, bd, rmd, rvd, epsd, momd):
        C = x3.shape[1]
        f32 = dict(dtype=torch.float32, device=x3.device)
        v3 = [torch.empty(C, **f32) for _ in range(4)]
        vd = [torch.empty(C, **f32) for _ in range(4)]
        z = torch.empty_like(x3, memory_format=torch.channels_last)
        mask = torch.empty(x3.numel() // 8, dtype=torch.uint8, device=x3.device)
        native().bn_dual_forward(part3, part3.shape[2], partd, partd.shape[2], x3, xd, z, mask, w3, b3, rm3, rv3, *v3,
                                 wd, bd, rmd, rvd, *vd, C, float(eps3), float(mom3), float(epsd), float(momd))
        ctx.C = C
        ctx.save_for_backward(x3, xd, mask, w3, v3[0], v3[1], wd, vd[0], vd[1])
        ctx.bngrad = BNGradTap(x3, mask, v3[0], v3[1], v3[2], v3[3])
        z._hipps_bngrad = ctx.bngrad
        return z

    @staticmethod
    def backward(ctx, dz):
        x3, xd, mask, w3, mean3, invstd3, wd, meand, invstdd = ctx.saved_tensors
        dz = dz.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bg, ctx.bngrad = ctx.bngrad, None
        part3 = bg.part if bg is not None else None
        if bg is not None:
            bg.part = None
        dx3 = torch.empty_like(x3, memory_format=torch.channels_last)
        dxd = torch.empty_like(xd, memory_format=torch.channels_last)
        dw3, db3, dwd, dbd = (torch.empty_like(w3) for _ in range(4))
        native().bn_dual_backward(part3, 0 if part3 is None else part3.shape[2], dz, x3, xd, mask, w3, mean3, invstd3,
                                  wd, meand, invstdd, dx3, dxd, dw3, db3, dwd, dbd, ctx.C)
        return dx3, None, dw3, db3, None, None, None, None, dxd, None, dwd, dbd, None, None, None, None


def dual_bn_relu_ok(bn3, bnd, x3, xd) -> bool:
    """Can _DualBNRelu run relu(bn3(x3) + bnd(xd))?"""
    return (bn3.training and bnd.training and bn3.relu and not bnd.relu and bn3._fast_ok(x3, None) and
            bnd._fast_ok(xd, None) and x3.shape == xd.shape and bn3.weight.dtype == torch.float32 and
            bnd.weight.dtype == torch.float32)


def dual_bn_relu(bn3, x3, part3, bnd, xd, partd):
    """relu(bn3(x3) + bnd(xd)) with both BNs' statistics partials from their producers
    (callers check dual_bn_relu_ok first)."""
    bn3._nbt_pending += 1
    bnd._nbt_pending += 1
    return _DualBNRelu.apply(x3, part3, bn3.weight, bn3.bias, bn3.running_mean, bn3.running_var, bn3.eps,
                             bn3.momentum, xd, partd, bnd.weight, bnd.bias, bnd.running_mean, bnd.running_var,
                             bnd.eps, bnd.momentum)


def conv1x1_bn_input(conv: nn.Conv2d, x, tap=None, alias: bool = False, bn_grad: bool = False):
    """The conv half of conv_bn for a 1x1 conv on the MFMA path: (y, part[, x_alias]) -- the conv
    output and the following BN's statistics partials, with the same tap / alias / S2Tap /
    BNGradTap wiring as conv_bn.  Callers check conv1x1_ok (and training) first."""
    s = conv.stride[0]
    own_tap = tap if s == 1 else None
    bg = getattr(x, "_hipps_bngrad", None) if bn_grad else None
    s2tap = S2Tap() if (alias and s == 1) else (getattr(x, "_hipps_s2tap", None) if s == 2 else None)
    outs = conv1x1_stats(x, conv.weight, s, own_tap, alias and s == 1, bg, s2tap)
    if own_tap is not None:
        own_tap.armed = True
    if alias and s == 1:
        outs[2]._hipps_s2tap = s2tap
    return outs


def fused_bn_act(x, weight, bias, running_mean, running_var, eps=1e-5, momentum=0.1, relu=True, residual=None,
                 part=None, res_tap=None):
    """Training-mode BN (+residual) (+ReLU) on a channels-last bf16 HIP tensor.  ``part``: the
    [2, C, nrb] partial statistics when the producer (conv1x1_stats) already reduced them.
    ``res_tap``: an armed ResidualTap -- the residual's gradient goes to its consumer instead
    of autograd (the residual input then receives no gradient from this op)."""
    return _FusedBNAct.apply(x, residual, weight, bias, running_mean, running_var, eps, momentum, relu, part,
                             res_tap)


class FusedBatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d with optional fused residual add and ReLU."""

    def __init__(self, num_features, relu: bool = False, fused: bool = True, **kw):
        super().__init__(num_features, **kw)
        self.relu = relu
        self.fused = fused
        # num_batches_tracked is only read when momentum is None; bumping the device buffer costs
        # one kernel launch per BN per step (53 per ResNet-50 step), so count on the host and fold
        # the count in whenever the state is read.
        self._nbt_pending = 0
        self.register_state_dict_pre_hook(lambda mod, *a, **k: mod.sync_num_batches_tracked())

    def sync_num_batches_tracked(self):
        if self._nbt_pending and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(self._nbt_pending)
        self._nbt_pending = 0

    def extra_repr(self):
        return super().extra_repr() + f", relu={self.relu}, fused={self.fused}"

    def _fast_ok(self, x, residual) -> bool:
        if not (self.fused and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
            return False
        C = x.shape[1]
        if C % 8 or C > 2048 or not self.affine or not x.is_contiguous(memory_format=torch.channels_last):
            return False
        if self.training and (not self.track_running_stats or self.momentum is None):
            return False
        if residual is not None and (residual.dtype != torch.bfloat16 or residual.shape != x.shape or
                                     not residual.is_contiguous(memory_format=torch.channels_last)):
            return False
        if x.numel() % 16:
            return False
        return True

    def forward(self, x, residual=None, stats=None, res_tap=None):
        if self._fast_ok(x, residual):
            if self.training:
                self._nbt_pending += 1
                tap = res_tap if (res_tap is not None and res_tap.armed and residual is not None) else None
                return fused_bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps,
                                    self.momentum, self.relu, residual, stats, tap)
            if not torch.is_grad_enabled() or not (x.requires_grad or (residual is not None and
                                                                       residual.requires_grad)):
                scale = self.weight / torch.sqrt(self.running_var + self.eps)
                shift = self.bias - self.running_mean * scale
                y = torch.empty_like(x, memory_format=torch.channels_last)
                native().bn_apply(x, residual, y, scale.float().contiguous(), shift.float().contiguous(),
                                  x.shape[1], self.relu)
                return y
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        if self.relu:
            y = F.relu(y)
        return y


def conv_bn(conv: nn.Conv2d, bn: FusedBatchNorm2d, x, residual=None, fuse: bool = True, tap=None, res_tap=None,
            alias: bool = False, bn_grad: bool = False):
    """bn(conv(x), residual): a 1x1 conv that feeds a training-mode fused BN runs as the MFMA GEMM
    with the BN statistics in its epilogue (one fewer pass over the conv output).

    Gradient fusion for residual blocks (see ResidualTap / _Conv1x1):
      tap      this conv's dgrad epilogue adds the tap's residual gradient (armed here when the
               MFMA path with its own dgrad is taken)
      res_tap  this BN routes its residual gradient into that tap (only if armed)
      alias    also return an alias of x whose gradient is summed in this conv's dgrad epilogue
               -> returns (out, x_alias)
      bn_grad  x is the output of a fused BN whose only gradient is this conv's input gradient
               (after the tap / alias sums): reduce that BN's backward statistics in the dgrad
               epilogue (BNGradTap)"""
    if fuse and bn.training and conv1x1_ok(conv, x):
        s = conv.stride[0]
        own_tap = tap if s == 1 else None
        bg = getattr(x, "_hipps_bngrad", None) if bn_grad else None
        # alias (conv1 of a downsample block): its dgrad takes the downsample's compact gradient;
        # stride 2 reading such an alias (the downsample): hand that gradient over (S2Tap)
        s2tap = S2Tap() if (alias and s == 1) else (getattr(x, "_hipps_s2tap", None) if s == 2 else None)
        outs = conv1x1_stats(x, conv.weight, s, own_tap, alias and s == 1, bg, s2tap)
        y, part = outs[0], outs[1]
        xa = outs[2] if len(outs) > 2 else x
        if alias and s == 1 and s2tap is not None:
            xa._hipps_s2tap = s2tap
        if own_tap is not None:
            own_tap.armed = True
        out = bn(y, residual, stats=part, res_tap=res_tap) if bn._fast_ok(y, residual) else bn(y, residual)
    else:
        xa = x
        out = bn(conv(x), residual)
    return (out, xa) if alias else out


class _GlobalAvgPool(torch.autograd.Function):
    """[N, C, H, W] channels-last -> [N, C] mean over H, W.  The backward writes the broadcast
    gradient g / (H*W) straight into an NHWC-contiguous tensor (C innermost: a vectorised copy),
    so the BatchNorm backward that consumes it needs no layout copy; autograd's default
    (expand of [N, C, 1, 1] + .contiguous(channels_last)) ran a strided 51 MB copy per step."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        return (g / (h * w)).view(n, 1, 1, c).expand(n, h, w, c).contiguous().permute(0, 3, 1, 2)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """torch.flatten(F.adaptive_avg_pool2d(x, 1), 1) for channels-last activations."""
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return _GlobalAvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def _pool_ok(m: nn.MaxPool2d, x: torch.Tensor) -> bool:
    def two(v):
        return tuple(v) if isinstance(v, (tuple, list)) else (v, v)

    if m.return_indices or m.ceil_mode or two(m.kernel_size) != (3, 3) or two(m.stride) != (2, 2):
        return False
    if two(m.padding) != (1, 1) or two(m.dilation) != (1, 1):
        return False
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0 and
            x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


class _MaxPool3s2(torch.autograd.Function):
    """3x3/s2/p1 max pool on channels-last bf16 (hipps/csrc/pool.hip): 4-bit argmax codes,
    gather-form backward (no atomics, no int64 index tensor)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        code = torch.empty(N * Ho * Wo * (C // 8), dtype=torch.int32, device=x.device)
        native().maxpool3s2_forward(x, y, code)
        ctx.save_for_backward(code)
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (code,) = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty(ctx.xshape, dtype=torch.bfloat16, device=dy.device, memory_format=torch.channels_last)
        native().maxpool3s2_backward(dy, code, dx)
        return dx


class _BNReluPool(torch.autograd.Function):
    """maxpool3s2(relu(bn(y))) for a training BatchNorm whose statistics arrive as producer partials
    (the stem conv's epilogue): finalize, then ONE pool pass that reads y and applies the BN + ReLU
    in its load (pool.hip, BN variant) -- the 411 MB BN output of a batch-256 stem is never written
    or re-read.  Backward: the pool's gather into dz, then the BN backward with the ReLU mask
    recomputed from y.  Values, tap codes and gradients are bit-identical to bn -> pool."""

    @staticmethod
    def forward(ctx, y, part, weight, bias, running_mean, running_var, eps, momentum):
        N, C, H, W = y.shape
        f32 = dict(dtype=torch.float32, device=y.device)
        mean, invstd = torch.empty(C, **f32), torch.empty(C, **f32)
        scale, shift = torch.empty(C, **f32), torch.empty(C, **f32)
        native().bn_finalize_partials(part, part.shape[2], N * H * W, weight, bias, running_mean, running_var, mean,
                                      invstd, scale, shift, C, float(eps), float(momentum))
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        out = torch.empty((N, C, Ho, Wo), dtype=torch.bfloat16, device=y.device, memory_format=torch.channels_last)
        code = torch.empty(N * Ho * Wo * (C // 8), dtype=torch.int32, device=y.device)
        native().maxpool3s2_forward(y, out, code, scale, shift)
        ctx.save_for_backward(y, code, weight, mean, invstd, scale, shift)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, code, weight, mean, invstd, scale, shift = ctx.saved_tensors
        dout = dout.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dz = torch.empty_like(y, memory_format=torch.channels_last)
        native().maxpool3s2_backward(dout, code, dz)
        dy = torch.empty_like(y, memory_format=torch.channels_last)
        dw, db = torch.empty_like(weight), torch.empty_like(weight)
        native().bn_backward(dz, y, None, MASK_X, weight, mean, invstd, scale, shift, dy, None, dw, db, y.shape[1],
                             None)
        return dy, None, dw, db, None, None, None, None


class _StemBlock(torch.autograd.Function):
    """pool(relu(bn(stem(x)))) for the ResNet stem in training mode, as one autograd node so the
    backward never materialises the pool's or the BatchNorm's input gradient (2 x 411 MB at batch
    256): csrc/stem.hip stem_bnpool_backward reduces the BN backward statistics on a recomputed
    pool gradient, then the stem weight gradient stages dy = BN-backward(pool-backward(dp)) straight
    into LDS.  Forward = _StemConv + _BNReluPool.  The image needs no gradient (checked by the
    caller)."""

    @staticmethod
    def forward(ctx, x, w_master, bn_w, bn_b, running_mean, running_var, eps, momentum):
        w = bf16_weight(w_master).contiguous(memory_format=torch.channels_last)
        n, _, h, wd = x.shape
        ho, wo = (h - 1) // 2 + 1, (wd - 1) // 2 + 1
        y = torch.empty((n, 64, ho, wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        part = torch.empty((2, 64, native().stem_mtiles(n, ho)), dtype=torch.float32, device=x.device)
        native().stem_forward(x, w, y, part)
        f32 = dict(dtype=torch.float32, device=x.device)
        mean, invstd = torch.empty(64, **f32), torch.empty(64, **f32)
        scale, shift = torch.empty(64, **f32), torch.empty(64, **f32)
        native().bn_finalize_partials(part, part.shape[2], n * ho * wo, bn_w, bn_b, running_mean, running_var, mean,
                                      invstd, scale, shift, 64, float(eps), float(momentum))
        hp, wp = (ho - 1) // 2 + 1, (wo - 1) // 2 + 1
        out = torch.empty((n, 64, hp, wp), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        code = torch.empty(n * hp * wp * 8, dtype=torch.int32, device=x.device)
        native().maxpool3s2_forward(y, out, code, scale, shift)
        ctx.wdtype = w_master.dtype
        ctx.save_for_backward(x, y, code, bn_w, mean, invstd, scale, shift)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y, code, bn_w, mean, invstd, scale, shift = ctx.saved_tensors
        dout = dout.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dbw, dbb = torch.empty_like(bn_w), torch.empty_like(bn_w)
        dw = torch.empty((64, 3, 7, 7), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
        native().stem_bnpool_backward(dout, code, y, x, bn_w, mean, invstd, scale, shift, dbw, dbb, dw,
                                      materialize_dy=_STEM_BWD_DY, quad=_STEM_QUAD)
        if ctx.wdtype != torch.float32:
            dw = dw.to(ctx.wdtype)
        return None, dw, dbw, dbb, None, None, None, None


def _pool_geom_ok(m) -> bool:
    def two(v):
        return tuple(v) if isinstance(v, (tuple, list)) else (v, v)

    return (not m.return_indices and not m.ceil_mode and two(m.kernel_size) == (3, 3) and two(m.stride) == (2, 2)
            and two(m.padding) == (1, 1) and two(m.dilation) == (1, 1))


def stem_block_ok(conv: nn.Conv2d, bn, pool, x: torch.Tensor) -> bool:
    """Can _StemBlock run conv -> bn (+ReLU) -> pool on this input?"""
    return (stem_ok(conv, x) and not x.requires_grad and torch.is_grad_enabled() and conv.training and
            isinstance(bn, FusedBatchNorm2d) and bn.training and bn.relu and bn.fused and bn.affine and
            bn.track_running_stats and bn.momentum is not None and bn.num_features == 64 and
            bn.weight.dtype == torch.float32 and isinstance(pool, MaxPool2d) and pool.fused and _pool_geom_ok(pool))


def stem_block(conv: nn.Conv2d, bn, pool, x: torch.Tensor) -> torch.Tensor:
    """pool(bn(conv(x))) on _StemBlock (callers check stem_block_ok first)."""
    bn._nbt_pending += 1
    xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    return _StemBlock.apply(xb, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps,
                            bn.momentum)


def bn_relu_maxpool(bn, pool, y, part=None):
    """pool(bn(y)) for a ReLU BatchNorm followed by the 3x3/s2 max pool (the ResNet stem); with the
    producer's partial statistics ``part`` and every piece on the fused kernels this is one pool
    pass (_BNReluPool), otherwise the two modules."""
    if (part is not None and bn.training and bn.relu and bn._fast_ok(y, None) and isinstance(pool, MaxPool2d)
            and pool.fused and _pool_ok(pool, y)):
        bn._nbt_pending += 1
        return _BNReluPool.apply(y, part, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum)
    if part is not None and bn.training and bn._fast_ok(y, None):
        return pool(bn(y, stats=part))
    return pool(bn(y))


class MaxPool2d(nn.MaxPool2d):
    """nn.MaxPool2d; the ResNet stem case (3x3, stride 2, pad 1) on channels-last bf16 HIP
    tensors runs the hipps kernels, everything else the PyTorch op."""

    def __init__(self, *a, fused: bool = True, **kw):
        super().__init__(*a, **kw)
        self.fused = fused

    def forward(self, x):
        if self.fused and _pool_ok(self, x):
            return _MaxPool3s2.apply(x)
        return super().forward(x)
