"""Flat parameter / gradient store and the bucket plan.

The reference keeps every parameter separate: one hook, one encode task, one pickle, two MPI
collectives and one optimizer call per tensor (ps.py:63-66, 140-190; 161 tensors for
ResNet-50).  hipps instead re-homes all parameters of an optimizer into ONE fp32 buffer and all
gradients into another (``param.data`` / ``param.grad`` become views), so that

  * the optimizer is one fused kernel per param group (not per tensor),
  * a bucket is a contiguous slice that a codec encodes with one launch,
  * a dense wire image (identity codec) is a linear copy of the flat buffer, which the fused
    aggregate+update kernel can read directly.

Every tensor's slot starts on a 16-element boundary (64 B fp32 / 32 B bf16), so every bucket
and group slice is 16-byte aligned for vector loads.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

ALIGN_ELEMS = 16


def _align(n: int, a: int = ALIGN_ELEMS) -> int:
    return (n + a - 1) // a * a


def _is_dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (any dim permutation, e.g. channels_last)."""
    if t.numel() <= 1:
        return True
    dims = sorted([(s, d) for d, s in enumerate(t.stride()) if t.size(d) != 1])
    expect = 1
    for s, d in dims:
        if s != expect:
            return False
        expect *= t.size(d)
    return True


@dataclass
class Slot:
    name: str
    param: torch.Tensor
    offset: int
    numel: int
    group: int


class FlatStore:
    """All params of ``groups`` in one flat fp32 buffer; grads in a second one."""

    def __init__(self, groups: Sequence[Sequence[torch.Tensor]], names: Optional[Dict[int, str]] = None,
                 device=None, dtype=torch.float32):
        names = names or {}
        self.slots: List[Slot] = []
        self.group_ranges: List[Tuple[int, int]] = []
        off = 0
        seen = set()
        for gi, params in enumerate(groups):
            g0 = off
            for p in params:
                if id(p) in seen:
                    raise ValueError("a parameter appears twice in the optimizer")
                seen.add(id(p))
                self.slots.append(Slot(names.get(id(p), f"param{len(self.slots)}"), p, off, p.numel(), gi))
                off = _align(off + p.numel())
            self.group_ranges.append((g0, off))
        self.numel = off
        if device is None:
            device = self.slots[0].param.device if self.slots else torch.device("cpu")
        self.device = torch.device(device)
        self.dtype = dtype
        self.data = torch.zeros(self.numel, dtype=dtype, device=self.device)
        # the flat gradient buffer is allocated on first use (``grad``): engines in 'gather' mode
        # with a dense codec gather autograd's gradients straight into the bucket messages and
        # never read it (Llama-3-8B: 32 GB per worker)
        self._grad: Optional[torch.Tensor] = None
        self.grad_mode = "flat"
        self._force_present = False
        self._stale = [False] * len(self.slots)  # flat grad view holds data from an earlier step
        for s in self.slots:
            p = s.param
            if p.dtype != dtype:
                raise TypeError(f"{s.name}: parameter dtype {p.dtype} != flat store dtype {dtype}; keep params fp32 "
                                "and use autocast for bf16 compute")
            src = p.data
            if not _is_dense(src):
                src = src.contiguous()
            v = self._view(self.data, s, src)
            v.copy_(src)
            p.data = v
            if p.grad is not None:  # keep a gradient the caller already computed
                g = p.grad
                p.grad = None
                gv = self._view(self.grad, s, p.data)
                gv.copy_(g)
                p.grad = gv

    @property
    def grad(self) -> torch.Tensor:
        if self._grad is None:
            self._grad = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        return self._grad

    @property
    def grad_allocated(self) -> bool:
        return self._grad is not None

    @staticmethod
    def _view(buf: torch.Tensor, s: Slot, like: torch.Tensor) -> torch.Tensor:
        seg = buf[s.offset:s.offset + s.numel]
        if like.is_contiguous():
            return seg.view(like.shape)
        return seg.as_strided(like.shape, like.stride())

    def param_view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        s = self.slots[i]
        return self._view(buf, s, s.param)

    def set_grad_mode(self, mode: str):
        """'flat': p.grad are views of self.grad; 'gather': autograd owns p.grad (engines gather)."""
        self.grad_mode = mode
        for s in self.slots:
            s.param.grad = None

    def attach_slot(self, i: int):
        """Flat mode: make ``param.grad`` the flat view, copying a stolen/assigned gradient in."""
        s = self.slots[i]
        p = s.param
        g = p.grad
        if g is None:
            return
        v = self._view(self.grad, s, p.data)
        if g.data_ptr() != v.data_ptr():
            if g.is_cuda:
                from hipps.ops.nn import wgrad_stream

                wgs = wgrad_stream(g.device)
                if wgs is not None:  # g may still be written on the weight-gradient side stream
                    torch.cuda.current_stream(g.device).wait_stream(wgs)
            v.copy_(g)
            p.grad = v

    def attach_grads(self):
        """Flat mode, at step time: every present gradient lives in its flat view; the view of a
        parameter without a gradient (``p.grad is None``) is zeroed so codecs read zeros there."""
        if self.grad_mode == "gather":
            return
        for i, s in enumerate(self.slots):
            if s.param.grad is None:
                if self._stale[i]:
                    self.grad[s.offset:s.offset + s.numel].zero_()
                    self._stale[i] = False
            else:
                self.attach_slot(i)
                self._stale[i] = True

    def presence(self) -> List[bool]:
        """Per slot: did the parameter get a gradient since the last zero_grad()?  torch
        semantics -- ``p.grad is not None`` (zero_grad(set_to_none=False) keeps zero grads, which
        count as present)."""
        if self._force_present:
            return [True] * len(self.slots)
        return [s.param.grad is not None for s in self.slots]

    def grads_attached(self) -> bool:
        return all(s.param.grad is not None and s.param.grad.data_ptr() ==
                   self.grad[s.offset:].data_ptr() for s in self.slots)

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics: ``set_to_none=True`` (default) -> ``p.grad = None`` (autograd then
        hands its gradient tensor over without an accumulate kernel, and parameters that get no
        gradient are skipped by the update); ``False`` -> zero-filled gradients that count as
        present."""
        self._force_present = not set_to_none
        if set_to_none or self.grad_mode == "gather":
            for s in self.slots:
                s.param.grad = None
            return
        self.grad.zero_()
        for i, s in enumerate(self.slots):
            s.param.grad = self._view(self.grad, s, s.param.data)
            self._stale[i] = False

    def enable_bf16_shadow(self):
        """Keep a flat bf16 copy of ``data`` that the hipps conv kernels read (ops.nn.bf16_weight)."""
        from ..ops import nn as hnn

        if getattr(self, "shadow", None) is None:
            self.shadow = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            hnn.register_weight_shadow(self.data, self.shadow)
            self._build_transposed_shadow()
        self.refresh_shadow()

    def _build_transposed_shadow(self):
        """Backward-operand bf16 copies refreshed with the shadow by one multi-matrix transpose
        kernel (flat.hip k_transpose_cast): [Cin, Cout] for every 1x1-conv weight (the input-
        gradient GEMM's B operand), rot180(W)^T as a channels-last [Cin, Cout, KH, KW] weight for
        every square KxK conv (stride-1 input gradient as a forward convolution, ops.nn._ConvKxK)
        and W^T [in, out] for each Linear weight marked by ops.nn.mark_transposed_reader."""
        from ..ops import _native
        from ..ops import nn as hnn

        self.tshadow = self._tiles = None
        self._tile_ranges = {}
        if self.device.type != "cuda" or not _native.available():
            return
        mats, off = [], 0
        for s in self.slots:
            p = s.param
            if p.dim() == 4 and p.shape[2] == p.shape[3] and _is_dense(p.data) and \
                    (p.shape[2] == 1 or p.is_contiguous(memory_format=torch.channels_last)):
                mats.append((s, off))
                off += s.numel
            elif p.dim() == 2 and getattr(p, "reads_bf16_shadow_t", False) and p.is_contiguous():
                # a Linear weight [out, in] whose input-gradient GEMM runs on gemm2 (ops.nn
                # mark_transposed_reader): [in, out]
                mats.append((s, off))
                off += s.numel
        if not mats:
            return
        self.tshadow = torch.empty(off, dtype=torch.bfloat16, device=self.device)
        rows = []
        for s, toff in mats:
            R, C, KH, KW = s.param.shape if s.param.dim() == 4 else (*s.param.shape, 1, 1)
            T = KH * KW
            for kh in range(KH):
                for kw in range(KW):
                    so = s.offset + (kh * KW + kw) * C
                    do = toff + ((KH - 1 - kh) * KW + (KW - 1 - kw)) * R
                    rows += [(so, do, R, C, r0, c0, T * C, T * R) for r0 in range(0, R, 64) for c0 in range(0, C, 64)]
            seg = self.tshadow[toff:toff + s.numel]
            view = seg.view(C, R) if T == 1 else seg.as_strided((C, R, KH, KW), (T * R, 1, KW * R, R))
            hnn.register_transposed_weight(s.param, view)
        self._tiles = torch.tensor(rows, dtype=torch.int64).to(self.device)

    def disable_bf16_shadow(self):
        from ..ops import nn as hnn

        if getattr(self, "shadow", None) is not None:
            hnn.unregister_weight_shadow(self.shadow)
            if getattr(self, "tshadow", None) is not None:
                for s in self.slots:
                    hnn.unregister_transposed_weight(s.param)
            self.shadow = self.tshadow = self._tiles = None
            self._tile_ranges = {}

    def refresh_shadow(self, lo: int = 0, hi: Optional[int] = None, cast: bool = True):
        """Re-cast the bf16 shadows of ``data[lo:hi]`` (default: all) on the current stream; a
        range must start and end at slot boundaries (ps_async pull_overlap refreshes the two
        halves of a split pull on their own streams).  ``cast=False``: the flat shadow was already
        written (by the pull kernel that adopted ``data``); only the transposed copies are rebuilt."""
        if getattr(self, "shadow", None) is None:
            return
        full = lo == 0 and (hi is None or hi >= self.numel)
        hi = self.numel if hi is None else hi
        if cast:
            self.shadow[lo:hi].copy_(self.data[lo:hi])  # one vectorized cast kernel
        if getattr(self, "tshadow", None) is not None:
            from ..ops._native import native

            tiles = self._tiles if full else self._tiles_in(lo, hi)
            if tiles is not None and tiles.numel():
                native().transpose_cast(self.data, self.tshadow, tiles)

    def _tiles_in(self, lo: int, hi: int):
        """The transpose tiles whose source matrix lies in data[lo:hi] (cached per range)."""
        cache = self.__dict__.setdefault("_tile_ranges", {})
        if (lo, hi) not in cache:
            t = self._tiles
            sel = (t[:, 0] >= lo) & (t[:, 0] < hi)
            cache[(lo, hi)] = t[sel].contiguous()
        return cache[(lo, hi)]

    # ---- per-step "parameter has a gradient" masks (ps.py:178-179 skip semantics) -----------
    @property
    def nchunks(self) -> int:
        return self.numel // ALIGN_ELEMS  # numel is a multiple of 16

    def chunk_slots(self) -> torch.Tensor:
        """Device int32 [nchunks]: the slot owning each 16-element chunk (static, cached)."""
        cs = getattr(self, "_chunk_slots", None)
        if cs is None:
            counts = torch.tensor([(_align(s.offset + s.numel) - s.offset) // ALIGN_ELEMS for s in self.slots],
                                  dtype=torch.int64)
            cs = torch.repeat_interleave(torch.arange(len(self.slots), dtype=torch.int32), counts)
            if cs.numel() < self.nchunks:  # trailing group padding (never updated)
                cs = torch.cat([cs, cs.new_zeros(self.nchunks - cs.numel())])
            cs = cs.to(self.device)
            self._chunk_slots = cs
        return cs

    def chunk_mask(self, slot_present: torch.Tensor) -> torch.Tensor:
        """uint8 [nslots] (device) -> uint8 [nchunks] chunk mask for the fused update kernels."""
        return slot_present.to(self.device, torch.uint8).index_select(0, self.chunk_slots())

    def group_slice(self, buf: torch.Tensor, gi: int) -> torch.Tensor:
        a, b = self.group_ranges[gi]
        return buf[a:b]

    def new_buffer(self, dtype=None, zero=True) -> torch.Tensor:
        f = torch.zeros if zero else torch.empty
        return f(self.numel, dtype=dtype or self.dtype, device=self.device)


GUARD_BYTES = 16
GUARD_BYTE = 0x29  # the reference's sentinel byte (mpi_comms.py:80)


@dataclass
class Bucket:
    index: int
    lo: int
    hi: int
    slot_ids: List[int]
    wire_offset: int = 0
    layout: object = None
    msg_nbytes: int = 0  # layout bytes + canary guard (debug_canary)

    @property
    def numel(self):
        return self.hi - self.lo


class BucketPlan:
    """Contiguous flat slices, filled in autograd (reverse registration) order.

    Buckets are ready in ``ready_order`` (the last layers' gradients first) but their messages are
    laid out in FLAT order inside the wire buffer, so a dense codec's wire buffer is a linear
    image of the flat gradient.
    """

    def __init__(self, store: FlatStore, codec, bucket_bytes: int = 64 << 20, guard: bool = False):
        self.store = store
        self.codec = codec
        self.guarded = bool(guard)
        cap = max(1, bucket_bytes // store.data.element_size())
        rev = list(range(len(store.slots)))[::-1]
        groups: List[List[int]] = []
        cur: List[int] = []
        cur_n = 0
        for i in rev:
            cur.append(i)
            cur_n += store.slots[i].numel
            if cur_n >= cap:
                groups.append(cur)
                cur, cur_n = [], 0
        if cur:
            groups.append(cur)
        # flat order: group with lowest offsets first
        spans = []
        for ids in groups:
            lo = min(store.slots[i].offset for i in ids)
            hi = max(_align(store.slots[i].offset + store.slots[i].numel) for i in ids)
            spans.append((lo, hi, sorted(ids)))
        spans.sort()
        # make spans tile [0, numel) exactly (alignment padding belongs to the preceding bucket)
        self.buckets: List[Bucket] = []
        for bi, (lo, hi, ids) in enumerate(spans):
            nxt = spans[bi + 1][0] if bi + 1 < len(spans) else store.numel
            self.buckets.append(Bucket(bi, lo if bi else 0, nxt, ids))
        woff = 0
        g = GUARD_BYTES if self.guarded else 0
        for b in self.buckets:
            b.layout = codec.layout(b.numel)
            b.wire_offset = woff
            b.msg_nbytes = b.layout.nbytes + g
            woff += b.msg_nbytes
        self.wire_nbytes = woff
        # the whole wire is one dense image of the flat gradient only without guards
        self.dense_ok = bool(codec.fusable) and not self.guarded
        self._gidx = {}
        self.ready_order = [b.index for b in reversed(self.buckets)]
        self.slot_bucket = {}
        for b in self.buckets:
            for i in b.slot_ids:
                self.slot_bucket[i] = b.index

    def views(self, wire: torch.Tensor, bi: int):
        b = self.buckets[bi]
        return b.layout.views(wire[b.wire_offset:b.wire_offset + b.layout.nbytes])

    def message(self, wire: torch.Tensor, bi: int) -> torch.Tensor:
        """Bucket bi's message bytes (layout + guard) inside a whole-wire buffer."""
        b = self.buckets[bi]
        return wire[b.wire_offset:b.wire_offset + b.msg_nbytes]

    def _guard_index(self, device) -> torch.Tensor:
        key = str(device)
        if key not in self._gidx:
            idx = [torch.arange(b.wire_offset + b.layout.nbytes, b.wire_offset + b.msg_nbytes) for b in self.buckets]
            self._gidx[key] = torch.cat(idx).to(device)
        return self._gidx[key]

    def fill_guards(self, wire: torch.Tensor):
        if self.guarded:
            wire[self._guard_index(wire.device)] = GUARD_BYTE

    def bad_guards(self, wire: torch.Tensor) -> torch.Tensor:
        """Per-bucket bool (device): canary overwritten in a whole-wire buffer."""
        g = wire[self._guard_index(wire.device)].view(len(self.buckets), GUARD_BYTES)
        return (g != GUARD_BYTE).any(dim=1)

    @staticmethod
    def bad_guard(msg: torch.Tensor, layout_nbytes: int) -> torch.Tensor:
        """Device bool: canary of ONE message buffer (layout + guard) overwritten."""
        return (msg[layout_nbytes:layout_nbytes + GUARD_BYTES] != GUARD_BYTE).any()

    def new_wire(self, device=None) -> torch.Tensor:
        return torch.empty(self.wire_nbytes, dtype=torch.uint8, device=device or self.store.device)

    def dense_image(self, wire: torch.Tensor) -> torch.Tensor:
        """For fusable (identity) codecs: the whole wire buffer as one flat tensor."""
        dt = self.buckets[0].layout.fields[0].dtype
        return wire[: self.wire_nbytes].view(dt)
