"""hipps' own RCCL communicator for the sync engines (``PSConfig.transport='rccl'``).

Wraps the native ``hipps._C.RcclComm`` (hipps/csrc/runtime/rccl.cpp): the communicator is
created from a unique id that rank 0 draws and the default torch.distributed group broadcasts,
and every collective is enqueued on the caller's HIP stream.  Compared to the torch process
group it adds what the PS engines need natively:

  * ``gather`` = one ``ncclGather`` (rccl.h:745) for the sync PS's gather-to-root;
  * ``all_gather_v`` = grouped send/recv into static per-rank offsets (no allgatherv in RCCL);
  * ``poll()`` = ``ncclCommGetAsyncError``: a lost peer raises instead of hanging;
  * ``abort()`` = ``ncclCommAbort``: the watchdog tears the communicator down before exiting;
  * ``gather_v`` = grouped receives at the root (exact per-rank counts, no padded slots).

``Engine.object_exchange`` moves the reference-style codec objects (ps.py:140-147 /
mpi_comms.py:150-163: a size round, then a variable-size all-gather) through ``all_gather_v`` /
``gather_v`` when ``transport='rccl'``.
"""
from __future__ import annotations

from typing import List, Optional

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

    @staticmethod
    def _stream(stream=None) -> int:
        return (stream or torch.cuda.current_stream()).cuda_stream

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        self.comm.all_gather(inp, out, self._stream(stream))

    def all_gather_v(self, out: torch.Tensor, inp: torch.Tensor, counts: List[int], displs: List[int], stream=None):
        self.comm.all_gather_v(inp, out, counts, displs, self._stream(stream))

    def gather_into(self, out: Optional[torch.Tensor], inp: torch.Tensor, dst: int = 0, stream=None):
        self.comm.gather(inp, out, dst, self._stream(stream))

    def gather_v(self, out: Optional[torch.Tensor], inp: torch.Tensor, counts: List[int], displs: List[int],
                 dst: int = 0, stream=None):
        self.comm.gather_v(inp, out, counts, displs, dst, self._stream(stream))

    def broadcast(self, t: torch.Tensor, src: int = 0, stream=None):
        self.comm.broadcast(t, src, self._stream(stream))

    def poll(self):
        """Raise if RCCL reported an asynchronous error (ncclCommGetAsyncError)."""
        code = self.comm.async_error()
        if code:
            raise RcclError(f"RCCL communicator failed: {self.comm.error_string(code)} (code {code})")

    def abort(self):
        self.comm.abort()

    def close(self):
        self.comm.destroy()
