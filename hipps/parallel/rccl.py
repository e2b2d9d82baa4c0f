"""hipps' own RCCL communicator for the sync engines (``PSConfig.transport='rccl'``).

Wraps the native ``hipps._C.RcclComm`` (hipps/csrc/runtime/rccl.cpp): the communicator is
created from a unique id that rank 0 draws and the default torch.distributed group broadcasts,
and every collective is enqueued on the caller's HIP stream.  Compared to the torch process
group it adds what the PS engines need natively:

  * ``gather`` = one ``ncclGather`` (rccl.h:745) for the sync PS's gather-to-root;
  * ``all_gather_v`` = grouped send/recv into static per-rank offsets (no allgatherv in RCCL);
  * ``poll()`` = ``ncclCommGetAsyncError``: a lost peer raises instead of hanging;
  * ``abort()`` = ``ncclCommAbort``: the watchdog tears the communicator down before exiting;
  * ``pair(i)`` = (PS, worker i) communicators from ``ncclCommSplit`` (rccl.h:290).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from hipps.ops._native import native


class RcclError(RuntimeError):
    pass


class RcclGroup:
    def __init__(self, world, device: torch.device):
        C = native()
        self.world = world
        self.device = device
        uid = [C.RcclComm.unique_id() if world.rank == 0 else None]
        if world.size > 1:
            dist.broadcast_object_list(uid, src=0)
        with torch.cuda.device(device):
            self.comm = C.RcclComm(uid[0], world.size, world.rank)
        self._pairs: Dict[int, object] = {}

    @staticmethod
    def _stream(stream=None) -> int:
        return (stream or torch.cuda.current_stream()).cuda_stream

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        self.comm.all_gather(inp, out, self._stream(stream))

    def all_gather_v(self, out: torch.Tensor, inp: torch.Tensor, counts: List[int], displs: List[int], stream=None):
        self.comm.all_gather_v(inp, out, counts, displs, self._stream(stream))

    def gather_into(self, out: Optional[torch.Tensor], inp: torch.Tensor, dst: int = 0, stream=None):
        self.comm.gather(inp, out, dst, self._stream(stream))

    def broadcast(self, t: torch.Tensor, src: int = 0, stream=None):
        self.comm.broadcast(t, src, self._stream(stream))

    def pair(self, i: int):
        """(PS = rank 0, worker i) communicator; collective: every rank calls pair(i) in order."""
        if i not in self._pairs:
            r = self.world.rank
            color = 0 if r in (0, i) else -1
            self._pairs[i] = self.comm.split(color, 0 if r == 0 else 1)
        return self._pairs[i]

    def poll(self):
        """Raise if RCCL reported an asynchronous error (ncclCommGetAsyncError)."""
        code = self.comm.async_error()
        if code:
            raise RcclError(f"RCCL communicator failed: {self.comm.error_string(code)} (code {code})")

    def abort(self):
        for p in self._pairs.values():
            if p is not None:
                p.abort()
        self.comm.abort()

    def close(self):
        for p in self._pairs.values():
            if p is not None:
                p.destroy()
        self._pairs = {}
        self.comm.destroy()
