"""Process-group plumbing (replaces the reference's module-level MPI.COMM_WORLD globals,
mpi_comms.py:11-13 / ps.py:71-73).

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL over xGMI on ROCm)
for device tensors or ``gloo`` for CPU plumbing.  Launch with ``python -m hipps.launch`` or
``torch.distributed.run`` (rendezvous on 127.0.0.1).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class World:
    rank: int = 0
    size: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: torch.device = torch.device("cpu")

    @property
    def distributed(self) -> bool:
        return self.size > 1

    @property
    def is_ps(self) -> bool:
        return self.rank == 0


def init_from_env(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> World:
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* if present; bind rank->GPU.
    ``timeout_s`` (default ``HIPPS_COMM_TIMEOUT_S`` or 600) bounds every collective of the
    default group; the engines add their own group with ``PSConfig.comm_timeout_s``."""
    if timeout_s is None:
        timeout_s = float(os.environ.get("HIPPS_COMM_TIMEOUT_S", "600"))
    backend = backend or os.environ.get("HIPPS_BACKEND") or None  # e.g. gloo to rehearse N ranks on 1 GPU
    rank = int(os.environ.get("RANK", "0"))
    size = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if size > 1 and not dist.is_initialized():
        be = backend or ("nccl" if use_gpu else "gloo")
        if be == "nccl" and torch.cuda.device_count() < size:
            raise RuntimeError(f"nccl needs one GPU per rank ({size} ranks, {torch.cuda.device_count()} GPUs); "
                               "set HIPPS_BACKEND=gloo to share a GPU")
        kw = {}
        if be == "nccl" and use_gpu:
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(be, rank=rank, world_size=size, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return current()


def current() -> World:
    if dist.is_available() and dist.is_initialized():
        be = dist.get_backend()
        dev = torch.device("cuda", torch.cuda.current_device()) if be == "nccl" else torch.device("cpu")
        return World(dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", dist.get_rank())), be,
                     dev)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return World(0, 1, 0, None, dev)


def barrier(world: Optional[World] = None):
    w = world or current()
    if w.size > 1:
        if w.backend == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, world: World, group=None):
    """out[W * n] <- concat_w inp_w   (one collective; gloo falls back to list all_gather)."""
    if world.size == 1:
        out[: inp.numel()].copy_(inp)
        return
    if world.backend == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        n = inp.numel()
        dist.all_gather([out[w * n:(w + 1) * n] for w in range(world.size)], inp, group=group)


def gather_into(out: Optional[torch.Tensor], inp: torch.Tensor, world: World, dst: int = 0, group=None):
    """Root receives concat_w inp_w into out (reference igather, mpi_comms.py:60-93)."""
    if world.size == 1:
        out[: inp.numel()].copy_(inp)
        return
    n = inp.numel()
    lst = [out[w * n:(w + 1) * n] for w in range(world.size)] if world.rank == dst else None
    dist.gather(inp, gather_list=lst, dst=dst, group=group)


def broadcast(t: torch.Tensor, world: World, src: int = 0, group=None):
    if world.size > 1:
        dist.broadcast(t, src=src, group=group)


def all_gather_v(out: torch.Tensor, inp: torch.Tensor, counts, world: World, group=None):
    """Variable-size all-gather (reference Iallgatherv, mpi_comms.py:160-163): rank r's ``counts[r]``
    elements land at ``out[sum(counts[:r]):]``; exactly the counted bytes move (pairwise
    isend/irecv: RCCL pair channels on GPU, gloo on CPU)."""
    displs = [0]
    for c in counts[:-1]:
        displs.append(displs[-1] + c)
    me = world.rank
    out[displs[me]:displs[me] + counts[me]].copy_(inp)
    if world.size == 1:
        return
    ops = []
    for r in range(world.size):
        if r == me:
            continue
        if counts[me]:
            ops.append(dist.P2POp(dist.isend, inp, r, group=group))
        if counts[r]:
            ops.append(dist.P2POp(dist.irecv, out[displs[r]:displs[r] + counts[r]], r, group=group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def gather_v(out: Optional[torch.Tensor], inp: torch.Tensor, counts, world: World, dst: int = 0, group=None):
    """Variable-size gather to ``dst`` (reference Igatherv, mpi_comms.py:88, with exact counts
    instead of padded slots)."""
    me = world.rank
    if me != dst:
        if counts[me]:
            dist.send(inp, dst, group=group)
        return
    displs = [0]
    for c in counts[:-1]:
        displs.append(displs[-1] + c)
    out[displs[me]:displs[me] + counts[me]].copy_(inp)
    works = [dist.irecv(out[displs[r]:displs[r] + counts[r]], r, group=group)
             for r in range(world.size) if r != me and counts[r]]
    for w in works:
        w.wait()
