"""Gradient codecs: the reference's pluggable ``code`` object (ps.py:57, 65-66, 94, 165-166).

The reference calls an external ``codings`` package: ``code.encode(grad)`` in a pool thread,
``pickle`` + ``blosc`` the result on the host, all-gathers the bytes, sets ``code.codes`` and
calls ``code.decode(c, cuda=...)`` per rank.  Here a codec owns a *fixed device wire layout*
per flat bucket, so encode is one (or a few) kernel launches writing straight into the comm
buffer and decode is fused into the PS/optimizer accumulation:

    layout(n)                       -> WireLayout (16-byte aligned fields, static size)
    encode_into(x, views, state)    -> writes the message for flat f32 gradient x
    accumulate(msgs, acc, ...)      -> acc (+)= sum_w decode(msg_w), rank order
    dense_source(views)             -> (fusable codecs) a tensor the fused optimizer reads directly

The reference's object API (``encode(grad) -> code``, ``decode(code, cuda=False)``, ``codes``)
is kept on top for drop-in use (see :class:`Codec`).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from hipps import ops

ALIGN = 16


def _align(x: int, a: int = ALIGN) -> int:
    return (x + a - 1) // a * a


@dataclass(frozen=True)
class Field:
    name: str
    dtype: torch.dtype
    numel: int
    offset: int

    @property
    def nbytes(self) -> int:
        return self.numel * torch.empty((), dtype=self.dtype).element_size()


class WireLayout:
    """Static byte layout of one message: fields at 16-byte aligned offsets."""

    def __init__(self, fields: Sequence[Tuple[str, torch.dtype, int]]):
        off = 0
        fs = []
        for name, dt, n in fields:
            off = _align(off)
            f = Field(name, dt, int(n), off)
            fs.append(f)
            off += f.nbytes
        self.fields: List[Field] = fs
        self.nbytes = _align(off)

    def views(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        assert buf.dtype == torch.uint8 and buf.numel() >= self.nbytes, (buf.dtype, buf.numel(), self.nbytes)
        return {f.name: buf[f.offset:f.offset + f.nbytes].view(f.dtype) for f in self.fields}

    def __repr__(self):
        return "WireLayout(%s, nbytes=%d)" % (", ".join(f"{f.name}:{f.dtype}x{f.numel}" for f in self.fields),
                                             self.nbytes)


class Codec:
    """Base codec.  Subclasses define layout/encode_into/accumulate."""

    name = "codec"
    fusable = False  # True if dense_source() exists (decode == dtype cast)
    lossless = False

    def __init__(self):
        self.codes = None  # reference API: engine sets the list of all ranks' codes (ps.py:165)
        self._seed = 0
        self._object_state: dict = {}

    # ---- flat-bucket interface -----------------------------------------------------------
    def layout(self, n: int) -> WireLayout:
        raise NotImplementedError

    def init_state(self, n: int, device) -> dict:
        return {}

    def encode_into(self, x: torch.Tensor, views: Dict[str, torch.Tensor], state: dict) -> None:
        raise NotImplementedError

    def accumulate(self, msgs: Sequence[Dict[str, torch.Tensor]], acc: torch.Tensor, gscale: float = 1.0,
                   accumulate: bool = False, acquire: bool = False) -> None:
        """acc (+)= gscale * sum of the decoded messages, in order.  ``acquire``: some message was
        written into this device's memory by another GPU (a remote worker's async-PS mailbox
        slot), so the decode kernels acquire at system scope before reading it."""
        raise NotImplementedError

    def dense_source(self, views: Dict[str, torch.Tensor]) -> torch.Tensor:
        raise NotImplementedError

    def push_copy(self, layout: "WireLayout", src: torch.Tensor, dst: torch.Tensor) -> bool:
        """Copy one message for the async PS push; codecs with a device-side count move only the
        used part.  Returns False to let the caller do a plain copy."""
        return False

    def used_bytes(self, layout: "WireLayout", msg: torch.Tensor) -> int:
        """Bytes of ``msg`` that carry information (host read for variable-size codecs)."""
        return layout.nbytes

    def nbytes(self, n: int) -> int:
        return self.layout(n).nbytes

    # ---- reference object API (ps.py:94, 165-166) ----------------------------------------
    def encode(self, grad: torch.Tensor, key=None, **kw) -> dict:
        """Reference object API.  Pass ``key`` (e.g. the parameter name) to keep per-tensor
        codec state such as error-feedback residuals across calls."""
        g = grad.detach().reshape(-1).float().contiguous()
        if g.data_ptr() % ALIGN:
            g = g.clone()
        lay = self.layout(g.numel())
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device=g.device)
        views = lay.views(buf)
        if key is None:
            st = self.init_state(g.numel(), g.device)
            st.pop("resid", None)
        else:
            st = self._object_state.setdefault(key, self.init_state(g.numel(), g.device))
        self.encode_into(g, views, st)
        return {"codec": self.name, "shape": tuple(grad.shape), "n": g.numel(), "buf": buf}

    def decode(self, code: dict, cuda: bool = False) -> torch.Tensor:
        buf = code["buf"]
        if cuda and not buf.is_cuda:
            buf = buf.cuda(non_blocking=True)
        lay = self.layout(code["n"])
        acc = torch.empty(code["n"], dtype=torch.float32, device=buf.device)
        self.accumulate([lay.views(buf)], acc, 1.0, False)
        return acc.view(code["shape"])

    def next_seed(self) -> int:
        self._seed += 1
        return self._seed


class Identity(Codec):
    """Dense pass-through; wire dtype fp32 (exact) or bf16 (2x fewer bytes)."""

    fusable = True

    def __init__(self, wire_dtype: torch.dtype = torch.float32):
        super().__init__()
        assert wire_dtype in (torch.float32, torch.bfloat16)
        self.wire_dtype = wire_dtype
        self.lossless = wire_dtype == torch.float32
        self.name = "fp32" if wire_dtype == torch.float32 else "bf16"

    def layout(self, n):
        return WireLayout([("x", self.wire_dtype, n)])

    def encode_into(self, x, views, state):
        ops.convert(x, views["x"])

    def accumulate(self, msgs, acc, gscale=1.0, accumulate=False, acquire=False):
        ops.aggregate([m["x"] for m in msgs], acc, gscale, accumulate, acquire)

    def dense_source(self, views):
        return views["x"]


class Int8(Codec):
    """Per-256-block absmax int8 (QSGD-style), optional stochastic rounding and error feedback."""

    name = "int8"

    def __init__(self, stochastic: bool = False, error_feedback: bool = True):
        super().__init__()
        self.stochastic = stochastic
        self.error_feedback = error_feedback

    def layout(self, n):
        return WireLayout([("scales", torch.float32, (n + ops.QBLOCK - 1) // ops.QBLOCK), ("q", torch.int8, n)])

    def init_state(self, n, device):
        return {"resid": torch.zeros(n, dtype=torch.float32, device=device)} if self.error_feedback else {}

    def encode_into(self, x, views, state):
        ops.q8_encode(x, state.get("resid"), views["q"], views["scales"], self.stochastic, self.next_seed())

    def accumulate(self, msgs, acc, gscale=1.0, accumulate=False, acquire=False):
        ops.q8_aggregate([m["q"] for m in msgs], [m["scales"] for m in msgs], acc, gscale, accumulate, acquire)


class TopK(Codec):
    """Exact magnitude top-k (k = ceil(ratio*n)), ascending int32 indices + f32/bf16 values."""

    name = "topk"

    def __init__(self, ratio: float = 0.01, value_dtype: torch.dtype = torch.float32, error_feedback: bool = True):
        super().__init__()
        assert 0 < ratio <= 1
        self.ratio = ratio
        self.value_dtype = value_dtype
        self.error_feedback = error_feedback

    def k_of(self, n: int) -> int:
        return max(1, min(n, int(math.ceil(self.ratio * n))))

    def layout(self, n):
        k = self.k_of(n)
        return WireLayout([("idx", torch.int32, k), ("val", self.value_dtype, k)])

    def init_state(self, n, device):
        st = {}
        if self.error_feedback:
            st["resid"] = torch.zeros(n, dtype=torch.float32, device=device)
        if device is not None and torch.device(device).type == "cuda":
            st["ws"] = torch.zeros(ops.topk_workspace_bytes(n, self.k_of(n)), dtype=torch.uint8, device=device)
        return st

    def encode_into(self, x, views, state):
        ops.topk_encode(x, state.get("resid"), views["idx"].numel(), views["idx"], views["val"], state.get("ws"))

    def accumulate(self, msgs, acc, gscale=1.0, accumulate=False, acquire=False):
        if not accumulate:
            acc.zero_()
        for m in msgs:  # rank order; one message has unique indices
            ops.topk_accumulate(m["idx"], m["val"], acc, gscale, acquire)


class TopKInt8(TopK):
    """Top-k values further quantized to int8 (one scale per 256 selected values)."""

    name = "topk_int8"

    def layout(self, n):
        k = self.k_of(n)
        return WireLayout([("idx", torch.int32, k), ("scales", torch.float32, (k + ops.QBLOCK - 1) // ops.QBLOCK),
                           ("q", torch.int8, k)])

    def init_state(self, n, device):
        st = super().init_state(n, device)
        st["vals"] = torch.empty(self.k_of(n), dtype=torch.float32, device=device)
        return st

    def encode_into(self, x, views, state):
        resid = state.get("resid")
        ops.topk_encode(x, resid, views["idx"].numel(), views["idx"], state["vals"], state.get("ws"))
        ops.q8_encode(state["vals"], None, views["q"], views["scales"], False, 0)
        if resid is not None:
            ops.topk_q8_residual(views["idx"], state["vals"], views["q"], views["scales"], resid)

    def accumulate(self, msgs, acc, gscale=1.0, accumulate=False, acquire=False):
        if not accumulate:
            acc.zero_()
        for m in msgs:
            ops.topk_q8_accumulate(m["idx"], m["q"], m["scales"], acc, gscale, acquire)


class Threshold(Codec):
    """Variable-size sparsification: every |g| > tau (ascending indices), at most
    ceil(max_ratio*n) of them.  The message has a static CAPACITY but a data-dependent COUNT
    stored in a device-side header that the decode kernel reads -- the "unknown-size" path of
    README.md:30-31 without a size round trip or a host sync."""

    name = "threshold"

    def __init__(self, tau: float = 1e-3, max_ratio: float = 0.05, value_dtype: torch.dtype = torch.float32,
                 error_feedback: bool = True):
        super().__init__()
        self.tau = float(tau)
        self.max_ratio = max_ratio
        self.value_dtype = value_dtype
        self.error_feedback = error_feedback

    def cap_of(self, n: int) -> int:
        return max(1, min(n, int(math.ceil(self.max_ratio * n))))

    def layout(self, n):
        k = self.cap_of(n)
        return WireLayout([("count", torch.int32, 4), ("idx", torch.int32, k), ("val", self.value_dtype, k)])

    def init_state(self, n, device):
        st = {}
        if self.error_feedback:
            st["resid"] = torch.zeros(n, dtype=torch.float32, device=device)
        if device is not None and torch.device(device).type == "cuda":
            st["ws"] = torch.zeros(ops.topk_workspace_bytes(n, self.cap_of(n)), dtype=torch.uint8, device=device)
        return st

    def encode_into(self, x, views, state):
        ops.thresh_encode(x, state.get("resid"), self.tau, views["count"], views["idx"], views["val"], state.get("ws"))

    def accumulate(self, msgs, acc, gscale=1.0, accumulate=False, acquire=False):
        if not accumulate:
            acc.zero_()
        for m in msgs:
            ops.thresh_accumulate(m["count"], m["idx"], m["val"], acc, gscale, acquire)

    @staticmethod
    def count(views) -> int:
        """Host read of a message's element count (diagnostics only; forces a sync)."""
        return int(views["count"][0])

    def push_copy(self, layout, src, dst) -> bool:
        if not src.is_cuda:
            return False
        f = {fl.name: fl for fl in layout.fields}
        ops.native().copy_counted(src, dst, f["idx"].offset, f["val"].offset,
                                  torch.empty((), dtype=self.value_dtype).element_size(), f["idx"].numel)
        return True

    def used_bytes(self, layout, msg) -> int:
        f = {fl.name: fl for fl in layout.fields}
        k = min(int(msg[:4].view(torch.int32)[0]), f["idx"].numel)
        return 16 + k * (4 + torch.empty((), dtype=self.value_dtype).element_size())


class ObjectCodec(Codec):
    """Adapter for the reference's codec plug-in contract (ps.py:57, 65-66, 94, 165-166): any
    object with ``encode(grad) -> code`` and ``decode(code, cuda=bool) -> tensor/ndarray``, whose
    ``codes`` attribute the engine sets to every contributing rank's code before decoding
    (ps.py:165).  Codes may be arbitrary picklable Python objects of unknown size (an SVD
    factorisation, QSGD levels + norms, ...) -- the "generic object / unknown size" path of
    README.md:24-31.

    One message per rank per step: ``{slot index: code}`` for every parameter that has a
    gradient, serialised with the zero-copy tensor frames of hipps.utils.serialization (+ the
    optional zlib level, mpi_comms.py:18-30).  Transport:
      allgather  size all-gather, then a payload all-gather of the max size (mpi_comms.py:144-174)
      ps_sync    size all-gather, then a gather to the PS (mpi_comms.py:60-117)
      ps_async   a length-prefixed blob in the worker's mailbox slot (capacity: object_slot_mb)
    Decode: per parameter, ``code.codes = [codes in rank order]``, decode each, check the shapes
    match (ps.py:172-175), sum in rank order (ps.py:176) into the fp32 flat gradient, then the
    fused optimizer kernel.  Encodes run in a thread pool like the reference's (ps.py:85)."""

    name = "object"
    is_object = True
    fusable = False
    HDR = 16  # int64 payload length + int64 reserved, then the payload

    def __init__(self, code, max_bytes: int = 0, level: int = 0, workers: int = 8):
        super().__init__()
        if not (callable(getattr(code, "encode", None)) and callable(getattr(code, "decode", None))):
            raise TypeError("an object codec needs encode(grad) and decode(code, cuda=...)")
        self.code = code
        self.max_bytes = int(max_bytes)
        self.level = int(level)
        self.workers = workers
        self.engine = None
        self._pool = None
        self.last_msg_bytes = 0
        self.last_packaged_bytes = 0

    def bind(self, engine):
        self.engine = engine

    def capacity(self, n: int) -> int:
        return self.max_bytes if self.max_bytes > 0 else 8 * n + (1 << 20)

    def layout(self, n):
        return WireLayout([("hdr", torch.int64, 2), ("blob", torch.uint8, self.capacity(n))])

    # ---- encode -----------------------------------------------------------------------------
    def encode_bytes(self, x: torch.Tensor) -> bytes:
        """Encode every present parameter of the bound store from flat gradient ``x`` (whole store)."""
        from concurrent.futures import ThreadPoolExecutor

        from hipps.utils.serialization import compress, dumps

        st = self.engine.store
        pres = st.presence()
        todo = [i for i, f in enumerate(pres) if f]
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=self.workers, thread_name_prefix="hipps-encode")

        def enc(i):
            s = st.slots[i]
            return i, self.code.encode(x[s.offset:s.offset + s.numel].view(s.param.shape))

        codes = dict(self._pool.map(enc, todo))
        raw = dumps(codes)
        packed = bytes(compress(raw, self.level)) if self.level else raw
        self.last_msg_bytes, self.last_packaged_bytes = len(raw), len(packed)
        return packed

    def encode_into(self, x, views, state):
        b = self.encode_bytes(x)
        state["bytes"] = b
        if getattr(self.engine, "object_wire", True):
            cap = views["blob"].numel()
            if len(b) > cap:
                raise ValueError(f"encoded message is {len(b)} bytes, the object codec slot holds {cap}; "
                                 "raise object_slot_mb")
            hdr = torch.tensor([len(b), 0], dtype=torch.int64)
            blob = torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else torch.empty(0, dtype=torch.uint8)
            views["hdr"].copy_(hdr)
            views["blob"][: len(b)].copy_(blob)

    # ---- decode -----------------------------------------------------------------------------
    def decode_messages(self, blobs: Sequence[bytes]) -> List[dict]:
        from hipps.utils.serialization import decompress, loads

        out = []
        for b in blobs:
            raw = decompress(b) if self.level else b
            out.append(loads(raw))
        return out

    def accumulate_codes(self, per_rank: Sequence[dict], acc: torch.Tensor, gscale: float = 1.0,
                         accumulate: bool = False) -> List[bool]:
        """acc (+)= gscale * sum over ranks of decode(code) per parameter; returns presence."""
        from hipps.utils.serialization import to_torch

        st = self.engine.store
        if not accumulate:
            acc.zero_()
        present = [False] * len(st.slots)
        cuda = acc.is_cuda
        for i, s in enumerate(st.slots):
            codes = [m[i] for m in per_rank if i in m]
            if not codes:
                continue
            present[i] = True
            self.code.codes = codes  # ps.py:165
            grads = []
            for c in codes:
                g = to_torch(self.code.decode(c, cuda=cuda))
                if not torch.is_tensor(g):
                    g = torch.as_tensor(g)
                grads.append(g.to(acc.device, torch.float32))
            if not all(g.numel() == s.numel for g in grads) or not all(g.shape == grads[0].shape for g in grads):
                raise ValueError(f"shapes not the same for {s.name}: {[tuple(g.shape) for g in grads]}")
            d = grads[0].reshape(-1).clone()
            for g in grads[1:]:  # rank order, like sum(grads) (ps.py:176)
                d += g.reshape(-1)
            if gscale != 1.0:
                d *= gscale
            acc[s.offset:s.offset + s.numel] += d
        return present

    def read_message(self, views, acquire: bool = False) -> bytes:
        hdr, blob = views["hdr"], views["blob"]
        if acquire and hdr.is_cuda:  # written by a peer GPU: stage through a system-scope acquire
            h = torch.empty(16, dtype=torch.uint8, device=hdr.device)
            ops.copy_acquire(hdr.view(torch.uint8), h)
            n = int(h.view(torch.int64)[0].item())
            m = min((n + 15) // 16 * 16, blob.numel())
            b = torch.empty(m, dtype=torch.uint8, device=blob.device)
            ops.copy_acquire(blob[:m], b)
            return b[:n].cpu().numpy().tobytes()
        n = int(hdr[0].item())
        return blob[:n].cpu().numpy().tobytes()

    def accumulate(self, msgs, acc, gscale=1.0, accumulate=False, acquire=False):
        self.last_present = self.accumulate_codes(
            self.decode_messages([self.read_message(v, acquire) for v in msgs]), acc, gscale, accumulate)


def get_codec(spec) -> Codec:
    """'fp32' | 'bf16' | 'int8' | 'int8_sr' | 'topk[:ratio]' | 'topk_bf16[:ratio]' | 'topk_int8[:ratio]' |
    'threshold[:tau[:max_ratio]]' | Codec instance | any object with encode()/decode() (the
    reference's ``codings`` contract, wrapped in :class:`ObjectCodec`)."""
    if spec is None:
        return Identity(torch.float32)
    if isinstance(spec, Codec):
        return spec
    if not isinstance(spec, str) and hasattr(spec, "encode") and hasattr(spec, "decode"):
        return ObjectCodec(spec)
    name, _, arg = str(spec).partition(":")
    name = name.lower()
    if name in ("fp32", "identity", "none"):
        return Identity(torch.float32)
    if name == "bf16":
        return Identity(torch.bfloat16)
    if name in ("int8", "qsgd"):
        return Int8(stochastic=False)
    if name in ("int8_sr", "qsgd_sr"):
        return Int8(stochastic=True)
    if name in ("threshold", "thresh"):
        tau, _, mr = arg.partition(":")
        return Threshold(tau=float(tau) if tau else 1e-3, max_ratio=float(mr) if mr else 0.05)
    ratio = float(arg) if arg else 0.01
    if name == "topk":
        return TopK(ratio)
    if name == "topk_bf16":
        return TopK(ratio, value_dtype=torch.bfloat16)
    if name == "topk_int8":
        return TopKInt8(ratio)
    raise ValueError(f"unknown codec {spec!r}")


__all__ = ["Codec", "Identity", "Int8", "TopK", "TopKInt8", "Threshold", "ObjectCodec", "WireLayout", "get_codec"]
