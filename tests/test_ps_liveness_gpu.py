"""Failure paths of the NATIVE PS loop (csrc/runtime/psloop.cpp), the loop production runs on the
GPU.  tests/test_ps_liveness_cpu.py covers the same paths for the Python
loop; here the ranks share one GPU (HIP-IPC mailboxes, device doorbells) and every case asserts
that the native loop served (``native_loop == 1``):

* rank 0's trainer parked longer than ``dead_after_s``: its own PS keeps serving the others
  (the loop never counts its own rank as dead, psloop.cpp dead_workers);
* the PS stops while a worker still trains: the worker raises within seconds, and the loop
  leaves the control block's error word set (should_stop / left_behind);
* the PS's heartbeat goes silent: the worker raises instead of waiting comm_timeout_s;
* a worker dies (HIPPS_FAULT=2:3:die): the PS keeps serving the other two, names the dead rank;
* a reader holds a publish buffer past ``dead_after_s``: the update that must rewrite it waits,
  counts ``reader_timeouts`` and goes on -- no hang.
"""
import os
import time

import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp

pytestmark = pytest.mark.gpu


def _opt(m, **kw):
    import hipps

    os.environ["HIPPS_NATIVE_PS"] = "1"
    return hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async", ps_granularity="bucket", **kw)


def _train(opt, m, rank, steps, s0=0):
    for s in range(s0, s0 + steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
        opt.step()


def _parked(rank, world, steps, park_s):
    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = _opt(m, dead_after_s=1.0, bucket_mb=0.0005, mailbox_slots=1)
    native = opt.engine._native is not None if rank == 0 else None
    done = 0
    for s in range(steps):
        if rank == 0 and s == 2:
            time.sleep(park_s)  # rank 0's trainer silent (no heartbeat) for > dead_after_s
        _train(opt, m, rank, 1, s)
        done += 1
    eng = opt.engine
    torch.cuda.synchronize()
    opt.close()
    return {"done": done, "stats": eng.ps_stats(), "native": native}


def test_native_parked_colocated_rank0_keeps_serving():
    out = run_world(_parked, 2, 8, 3.0, timeout=240)
    assert out[0]["native"] and out[0]["stats"]["native_loop"] == 1
    assert out[1]["done"] == 8 and out[0]["done"] == 8
    assert out[0]["stats"]["accumulated"] == 16 and out[0]["stats"]["updates"] == 8


def _stopped(rank, world, steps):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = _opt(m, bucket_mb=0.0005, mailbox_slots=1, comm_timeout_s=120.0)
    eng = opt.engine
    C = eng.C
    native = eng._native is not None if rank == 0 else None
    err, t_err = None, None
    for s in range(steps):
        if rank == 0 and s == 1:
            eng.ctl.store(C.F_PS_STOP, 0, 1)  # the PS leaves its loop while worker 1 still trains
            eng._thread.join(timeout=30)
        if rank == 1 and s >= 1:
            time.sleep(0.2)
        if rank == 0 and s >= 1:
            break
        t = time.time()
        try:
            _train(opt, m, rank, 1, s)
            torch.cuda.synchronize()
        except RuntimeError as e:
            err, t_err = str(e), time.time() - t
            break
    dist.barrier()
    code = eng.ctl.load(C.F_ERROR, 0)
    st = eng.ps_stats() if rank == 0 else {}
    try:
        opt.close()
    except Exception:
        pass
    return {"err": err, "t_err": t_err, "code": code, "native": native, "stats": st}


def test_native_ps_stop_makes_live_worker_raise():
    out = run_world(_stopped, 2, 40, timeout=240)
    assert out[0]["native"] and out[0]["stats"]["native_loop"] == 1
    assert out[0]["code"] == 2  # the loop left with a worker not stopped (psloop.cpp left_behind)
    assert out[1]["err"] is not None and "stopped serving" in out[1]["err"], out[1]
    assert out[1]["t_err"] < 10.0


def _silent(rank, world):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = _opt(m, bucket_mb=0.0005, mailbox_slots=1, dead_after_s=1.5, comm_timeout_s=120.0)
    eng = opt.engine
    C = eng.C
    native = eng._native is not None if rank == 0 else None
    if rank == 0:
        # the native loop disappears without a word (as a killed process would): stop it, then
        # clear the error word it leaves and let its heartbeat age
        eng.ctl.store(C.F_PS_STOP, 0, 1)
        eng._thread.join(timeout=30)
        eng.ctl.store(C.F_ERROR, 0, 0)
    dist.barrier()
    err, t_err = None, None
    if rank == 1:
        t = time.time()
        try:
            _train(opt, m, rank, 40)
            torch.cuda.synchronize()
        except RuntimeError as e:
            err, t_err = str(e), time.time() - t
    dist.barrier()
    try:
        opt.close()
    except Exception:
        pass
    return {"err": err, "t_err": t_err, "native": native}


def test_native_silent_ps_heartbeat_makes_worker_raise():
    out = run_world(_silent, 2, timeout=240)
    assert out[0]["native"]
    assert out[1]["err"] is not None and "silent" in out[1]["err"], out[1]
    assert out[1]["t_err"] < 15.0


def _faulty(rank, world, steps):
    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = _opt(m, dead_after_s=2.0)
    native = opt.engine._native is not None if rank == 0 else None
    _train(opt, m, rank, steps)
    torch.cuda.synchronize()
    eng = opt.engine
    if rank == 0:
        time.sleep(2.5)  # let the dead worker's heartbeat age past dead_after_s
    dead = eng.dead_workers() if rank == 0 else []
    opt.close()
    return {"stats": eng.ps_stats(), "dead": dead, "native": native}


def test_native_survives_dead_worker(monkeypatch):
    monkeypatch.setenv("HIPPS_FAULT", "2:3:die")
    out = run_world(_faulty, 3, 8, timeout=240)
    st = out[0]["stats"]
    assert out[0]["native"] and st["native_loop"] == 1
    # ranks 0, 1 pushed 8 steps each; rank 2 pushed 2 before dying -> 18 steps accumulated
    assert st["accumulated"] == 18 and st["updates"] == 18 // 3
    assert out[0]["dead"] == [2]


def _stuck_reader(rank, world, steps):
    """Rank 2 announces itself as a reader of bucket 0's initial publish (version 0) and never
    reads or releases it, then leaves training to ranks 0 and 1 (accumulate=1)."""
    import torch.distributed as dist

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = _opt(m, dead_after_s=1.0, accumulate=1, bucket_mb=0.0005)
    eng = opt.engine
    C = eng.C
    native = eng._native is not None if rank == 0 else None
    if rank == 2:
        eng.ctl.store(C.F_READING_B, 2 * C.ControlBlock.MAX_BUCKETS + 0, 0)
    dist.barrier()
    t0 = time.time()
    if rank != 2:
        _train(opt, m, rank, steps)
        torch.cuda.synchronize()
    t = time.time() - t0
    dist.barrier()
    if rank == 2:
        eng.ctl.store(C.F_READING_B, 2 * C.ControlBlock.MAX_BUCKETS + 0, -1)
    dist.barrier()
    opt.close()
    return {"stats": opt._last_engine_stats if rank == 0 else {}, "native": native, "t": t}


def test_native_reader_timeout_is_counted_not_hung():
    steps = 8
    out = run_world(_stuck_reader, 3, steps, timeout=300)
    st = out[0]["stats"]
    assert out[0]["native"] and st["native_loop"] == 1
    assert st["reader_waits"] >= 1 and st.get("reader_timeouts", 0) >= 1, st
    assert st["accumulated"] == 2 * steps  # every message of ranks 0 and 1 applied
    assert out[0]["t"] < 60 and out[1]["t"] < 60  # one dead_after_s wait, not a hang
