"""Host-side serialization: the reference's wire helpers, plus the zero-copy tensor format that
/root/reference/serialization.py set out to build (and never finished, serialization.py:25-30).

Reference behaviour kept (mpi_comms.py):
  compress/decompress   mpi_comms.py:18-30   (level 0 = framing only, like blosc clevel 0)
  to_np / to_torch      mpi_comms.py:32-58   (recursive over dict/list/map)
  format_for_send       mpi_comms.py:186-193 (returns (packaged, {'msg_bytes','packaged_bytes'}))
  trim_msg + sentinel   mpi_comms.py:80, 96-104

Differences (documented, deliberate):
  * c-blosc is not available; compression uses zlib behind a 16-byte frame header
    ('HPZ1', level, raw length).  'blosclz' is accepted as an alias; 'lz4'/'snappy' are
    rejected as in the reference (mpi_comms.py:22-24).
  * ``to_torch`` keeps the array dtype (the reference always produced float32 via
    ``torch.Tensor(ndarray)``, mpi_comms.py:48); pass ``dtype=torch.float32`` for the old cast.
  * ``dumps``/``loads``: tensors are NOT pickled.  The object tree is pickled with tensor
    placeholders and every tensor's raw bytes follow in one contiguous frame (16-byte aligned),
    so a receiver rebuilds tensors with ``torch.frombuffer`` (zero copy for CPU tensors).
"""
from __future__ import annotations

import io
import pickle
import struct
import warnings
import zlib
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

SENTINEL = b"\x29" * 32  # mpi_comms.py:80
_MAGIC = b"HPZ1"
_HDR = struct.Struct("<4sIQ")  # magic, level, raw length  (16 bytes)


def compress(msg, level: int = 0, name: str = "zlib") -> bytearray:
    """Frame (level 0) or zlib-compress ``msg``.  Returns a bytearray like the reference."""
    if name in ("lz4", "snappy"):
        raise ValueError("Do not specify lz4 or snappy (reference mpi_comms.py:22-24); use zlib/blosclz")
    if name not in ("zlib", "blosclz"):
        raise ValueError(f"unknown compressor {name!r}")
    raw = bytes(msg)
    body = raw if level == 0 else zlib.compress(raw, level)
    return bytearray(_HDR.pack(_MAGIC, level, len(raw)) + body)


def decompress(code) -> bytes:
    code = bytes(code)
    magic, level, n = _HDR.unpack_from(code)
    if magic != _MAGIC:
        raise ValueError("not a hipps compressed frame")
    body = code[_HDR.size:]
    out = body if level == 0 else zlib.decompress(body)
    if len(out) != n:
        raise ValueError("corrupt frame: length mismatch")
    return out


def to_np(d):
    """Tensors -> numpy (device tensors are copied to host), recursively (mpi_comms.py:32-43)."""
    if isinstance(d, torch.Tensor):
        t = d.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()
    if isinstance(d, dict):
        return {k: to_np(v) for k, v in d.items()}
    if isinstance(d, list):
        return [to_np(v) for v in d]
    if isinstance(d, tuple):
        return tuple(to_np(v) for v in d)
    if isinstance(d, map):
        return map(to_np, d)
    return d


def to_torch(d, cuda: bool = False, dtype=None):
    """numpy -> tensors (optionally on the current HIP device), recursively (mpi_comms.py:47-58)."""
    if isinstance(d, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(d))
        if dtype is not None:
            t = t.to(dtype)
        if cuda:
            t = t.cuda(non_blocking=True)
        return t
    if isinstance(d, dict):
        return {k: to_torch(v, cuda, dtype) for k, v in d.items()}
    if isinstance(d, list):
        return [to_torch(v, cuda, dtype) for v in d]
    if isinstance(d, tuple):
        return tuple(to_torch(v, cuda, dtype) for v in d)
    if isinstance(d, map):
        return map(lambda v: to_torch(v, cuda, dtype), d)
    return d


def format_for_send(obj, level: int = 0) -> Tuple[bytearray, Dict[str, int]]:
    """to_np -> pickle -> compress (mpi_comms.py:186-193)."""
    send = bytearray(pickle.dumps(to_np(obj)))
    packaged = compress(send, level)
    return packaged, {"msg_bytes": len(send), "packaged_bytes": len(packaged)}


def unformat(packaged, cuda: bool = False):
    return to_torch(pickle.loads(decompress(packaged)), cuda=cuda)


def trim_msg(msg) -> bytes:
    """Everything before the 32-byte 0x29 sentinel (mpi_comms.py:96-104)."""
    i = bytes(msg).find(SENTINEL)
    if i == -1:
        raise ValueError("trim_msg error; end of msg not found")
    return bytes(msg)[:i]


# ---- zero-copy tensor frames (the intent of reference serialization.py) --------------------
class _TRef:
    __slots__ = ("i",)

    def __init__(self, i):
        self.i = i

    def __reduce__(self):
        return (_TRef, (self.i,))


def _split(obj, tensors: List[torch.Tensor]):
    if isinstance(obj, torch.Tensor):
        tensors.append(obj)
        return _TRef(len(tensors) - 1)
    if isinstance(obj, dict):
        return {k: _split(v, tensors) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_split(v, tensors) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_split(v, tensors) for v in obj)
    return obj


def _join(obj, tensors):
    if isinstance(obj, _TRef):
        return tensors[obj.i]
    if isinstance(obj, dict):
        return {k: _join(v, tensors) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_join(v, tensors) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_join(v, tensors) for v in obj)
    return obj


_FRAME = struct.Struct("<4sQQ")  # 'HPT1', skeleton length, tensor count


def dumps(obj, level: int = 0) -> bytes:
    """Serialize without pickling tensor data: [frame | skeleton pickle | meta | raw tensor bytes]."""
    tensors: List[torch.Tensor] = []
    skel = pickle.dumps(_split(obj, tensors))
    metas, blobs, off = [], [], 0
    for t in tensors:
        c = t.detach().contiguous().cpu()
        # reshape(-1): a "contiguous" tensor with a size-1 last dim may still carry a stride != 1
        raw = c.reshape(-1).view(torch.uint8).numpy().tobytes() if c.numel() else b""
        if level:
            raw = zlib.compress(raw, level)
        off = (off + 15) // 16 * 16
        metas.append((str(c.dtype).replace("torch.", ""), tuple(c.shape), off, len(raw), level))
        blobs.append((off, raw))
        off += len(raw)
    meta = pickle.dumps(metas)
    head = _FRAME.pack(b"HPT1", len(skel), len(tensors)) + struct.pack("<Q", len(meta)) + skel + meta
    pad = (-len(head)) % 16
    out = bytearray(head + b"\0" * pad + b"\0" * off)
    base = len(head) + pad
    for o, raw in blobs:
        out[base + o:base + o + len(raw)] = raw
    return bytes(out)


def loads(buf, device=None):
    mv = memoryview(buf)
    magic, nskel, nt = _FRAME.unpack_from(mv)
    if magic != b"HPT1":
        raise ValueError("not a hipps tensor frame")
    p = _FRAME.size
    (nmeta,) = struct.unpack_from("<Q", mv, p)
    p += 8
    skel = pickle.loads(mv[p:p + nskel])
    p += nskel
    metas = pickle.loads(mv[p:p + nmeta])
    p += nmeta
    base = p + ((-p) % 16)
    tensors = []
    for dt, shape, off, n, level in metas:
        dtype = getattr(torch, dt)
        raw = mv[base + off: base + off + n]
        if level:
            raw = memoryview(zlib.decompress(raw))
        if n == 0 or len(raw) == 0:
            t = torch.empty(shape, dtype=dtype)
        else:
            with warnings.catch_warnings():  # read-only bytes input: tensors alias it (zero copy)
                warnings.simplefilter("ignore", UserWarning)
                t = torch.frombuffer(raw, dtype=torch.uint8).view(dtype).view(shape)
        if device is not None:
            t = t.to(device)
        tensors.append(t)
    return _join(skel, tensors)


# ---- debug helpers (ps.py:25-50, mpi_comms.py:176-184) -------------------------------------
def bytes_of(obj) -> int:
    """Payload bytes of tensors/arrays inside ``obj`` (fixes the reference's 1-D-only bug)."""
    if isinstance(obj, torch.Tensor):
        return obj.element_size() * obj.numel()
    if isinstance(obj, np.ndarray):
        return obj.nbytes
    if isinstance(obj, dict):
        return sum(bytes_of(v) for v in obj.values())
    if isinstance(obj, (list, tuple)):
        return sum(bytes_of(v) for v in obj)
    import sys

    return sys.getsizeof(obj)


def print_summary(flat_dict) -> str:
    parts = []
    for k, v in flat_dict.items():
        parts.append(f"{k}: {tuple(v.shape)}" if hasattr(v, "shape") else f"{k}: {v}")
    s = "    {" + ", ".join(parts) + "}"
    print(s)
    return s


def find_param(named_params, name):
    """Parameter by name (ps.py:44-48; names live in a dict since param.name is read-only)."""
    matches = [p for n, p in named_params if n == name]
    if len(matches) > 1:
        raise ValueError("More than one name found")
    if not matches:
        raise KeyError(name)
    return matches[0]
