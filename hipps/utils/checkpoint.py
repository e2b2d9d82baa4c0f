"""Checkpoint / resume.

The reference has none beyond torch.optim.Optimizer.state_dict() (its per-parameter state keys
are torch-compatible, ps.py:202-205, 223-234) and never saves ``MPI_PS.steps`` (ps.py:74).

Layout of a checkpoint directory (all files are plain tensors/ints: loadable with
``torch.load(..., weights_only=True)``):
  ps.pt          written by rank 0: parameters (the PS master in async mode), flat optimizer
                 state (momentum / Adam moments), per-group step counts, PS version, metadata
  rank<r>.pt     written by every rank: its codec state (error-feedback residuals), its worker
                 sequence numbers and (optionally) the model's buffers (BN running statistics)

``save``/``load`` are collective (every rank calls them).  In ps_async mode ``load`` must run
after constructing the optimizer and before the first ``step()``: the PS republishes the
restored master as the current version and every worker adopts it.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from hipps.parallel.dist import barrier, broadcast


def _cpu(d):
    return {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in d.items()}


def _buffers(model: torch.nn.Module) -> dict:
    for m in model.modules():  # fold host-side counters (FusedBatchNorm2d) into their buffers
        if hasattr(m, "sync_num_batches_tracked"):
            m.sync_num_batches_tracked()
    return {k: v.detach().cpu() for k, v in model.named_buffers()}


def save(opt, path: str, model: Optional[torch.nn.Module] = None, extra: Optional[dict] = None) -> None:
    os.makedirs(path, exist_ok=True)
    eng = opt.engine
    rank = opt.world.rank
    if hasattr(eng, "join_pull"):  # a split pull's late half may still be landing on a side stream
        eng.join_pull()
    # async PS: the PS thread is held between messages for the whole snapshot, so the master,
    # the optimizer state, the pending accumulator and the version belong to one PS state
    quiesce = getattr(eng, "quiesced", None)
    with (quiesce() if quiesce is not None else _nullctx()):
        es = eng.engine_state()
        master = es.pop("master", None)
        version = es.pop("version", None)
        acc = es.pop("acc", None)
        acc_count = es.pop("acc_count", 0)
        ps_acc, ps_seen = es.pop("ps_accumulated", None), es.pop("ps_seen", None)
        mine = {"engine": es}
        if model is not None:
            mine["buffers"] = _buffers(model)
        torch.save(mine, os.path.join(path, f"rank{rank}.pt"))
        if rank == 0:
            params = master if master is not None else opt.store.data.detach().cpu()
            ps = {"params": params, "flat_state": _cpu(opt.flat_state), "group_steps": list(opt._group_steps),
                  "steps": opt.steps, "mode": opt.mode, "codec": opt.codec.name, "numel": opt.store.numel,
                  "version": -1 if version is None else int(version),
                  "chunk_steps": None if opt.chunk_steps is None else opt.chunk_steps.detach().cpu()}
            if acc is not None:
                ps["acc"], ps["acc_count"] = acc, int(acc_count)
                # PS consumption at the snapshot: messages accumulated so far, per-worker seen seq
                ps["ps_accumulated"], ps["ps_seen"] = int(ps_acc), [int(v) for v in ps_seen]
            if extra:
                ps["extra"] = extra
            torch.save(ps, os.path.join(path, "ps.pt"))
    barrier(opt.world)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def load(opt, path: str, model: Optional[torch.nn.Module] = None) -> dict:
    ps = torch.load(os.path.join(path, "ps.pt"), map_location="cpu", weights_only=True)
    if ps["numel"] != opt.store.numel:
        raise ValueError(f"checkpoint has {ps['numel']} flat elements, optimizer has {opt.store.numel}")
    for k, v in ps["flat_state"].items():
        opt._ensure_state(k).copy_(v)
    opt._group_steps = list(ps["group_steps"])
    opt.steps = ps["steps"]
    cs = opt._csteps()
    if cs is not None:
        if ps.get("chunk_steps") is not None:
            cs.copy_(ps["chunk_steps"].to(cs.device))
        else:  # older checkpoint: per-group counts only (SGD: + the groups whose momentum started)
            opt.csteps_from_groups(cs, ps["mom_started"] if "mom_started" in ps else None)
    rank = opt.world.rank
    rp = os.path.join(path, f"rank{rank}.pt")
    mine = torch.load(rp, map_location="cpu", weights_only=True) if os.path.exists(rp) else {"engine": {}}
    if model is not None and "buffers" in mine:
        bufs = dict(model.named_buffers())
        for k, v in mine["buffers"].items():
            if k in bufs:
                bufs[k].copy_(v)
    es = dict(mine.get("engine", {}))
    if opt.mode == "ps_async":
        if rank == 0:
            es["master"] = ps["params"]
            es["version"] = max(0, ps["version"])
            if "acc" in ps:
                es["acc"], es["acc_count"] = ps["acc"], ps["acc_count"]
        opt.engine.load_engine_state(es)
    else:
        opt.store.data.copy_(ps["params"].to(opt.store.data.device))
        broadcast(opt.store.data, opt.world, 0)
        opt.engine.load_engine_state(es)
    opt.store.refresh_shadow()
    barrier(opt.world)
    return ps.get("extra", {})
