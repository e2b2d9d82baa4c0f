"""Async PS liveness and mailbox rendezvous, on CPU.

* a co-located rank 0 parked (in a barrier, a checkpoint, ...) for longer than ``dead_after_s``
  is never "dead" to its own PS: the other workers keep getting acks;
* a PS that stops while a worker still trains makes that worker raise within seconds, not after
  ``comm_timeout_s``;
* a mailbox import that does not return is reported by every rank together (the one that timed
  out raises ``IPCOpenTimeout`` with its thread diagnostic) instead of hanging or rebuilding;
* worker i maps only its own ring and the publish region;
* the default geometry of Llama-3-8B at W=8 fits rank 0's HBM budget (config 5).
"""
import math
import time

import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp


def _parked_rank0(rank, world, steps, park_s):
    import hipps

    m = _mlp()
    # 1-slot message words + small buckets: worker 1 needs the PS's acks every few messages
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async", dead_after_s=1.0, bucket_mb=0.0005,
                    mailbox_slots=1)
    t0 = time.time()
    done = 0
    for s in range(steps):
        if rank == 0 and s == 2:
            time.sleep(park_s)  # rank 0's trainer silent (no heartbeat) for > dead_after_s
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
        done += 1
    eng = opt.engine
    nb = len(eng.plan.buckets)
    opt.close()
    return {"done": done, "stats": eng.ps_stats(), "t": time.time() - t0, "nb": nb}


def test_parked_colocated_rank0_keeps_serving():
    """Worker 1 keeps pushing (and needs acks) while rank 0's trainer is silent for 3x
    dead_after_s: the PS must not treat its own rank as dead and stop."""
    out = run_world(_parked_rank0, 2, 8, 3.0, timeout=180)
    assert out[1]["done"] == 8 and out[0]["done"] == 8
    st = out[0]["stats"]
    assert st["accumulated"] == 16
    assert st["updates"] == 8  # M = W = 2 per version


def _ps_stopped(rank, world, steps):
    import torch.distributed as dist

    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async", bucket_mb=0.0005, mailbox_slots=1,
                    comm_timeout_s=120.0)
    eng = opt.engine
    C = eng.C
    err, t_err = None, None
    for s in range(steps):
        if rank == 0 and s == 1:
            eng.ctl.store(C.F_PS_STOP, 0, 1)  # the PS leaves its loop while worker 1 still trains
            eng._thread.join(timeout=30)
        if rank == 1 and s >= 1:
            time.sleep(0.2)
        if rank == 0 and s >= 1:
            break  # rank 0 stops training once its PS has stopped
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        t = time.time()
        try:  # (a hook-time push may raise from backward())
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
        except RuntimeError as e:
            err, t_err = str(e), time.time() - t
            break
    dist.barrier()
    try:
        opt.close()
    except Exception:
        pass
    return {"err": err, "t_err": t_err, "code": eng.ctl.load(C.F_ERROR, 0)}


def test_worker_raises_when_ps_stops_serving():
    out = run_world(_ps_stopped, 2, 40, timeout=180)
    assert out[0]["code"] == 2
    assert out[1]["err"] is not None and "stopped serving" in out[1]["err"], out[1]
    assert out[1]["t_err"] < 10.0  # not comm_timeout_s


def _ps_silent(rank, world):
    import torch.distributed as dist

    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async", bucket_mb=0.0005, mailbox_slots=1,
                    dead_after_s=1.5, comm_timeout_s=120.0)
    eng = opt.engine
    C = eng.C
    if rank == 0:
        # the PS thread disappears without a word (as a killed process would): stop its loop,
        # then clear the error word it leaves and let its liveness word age
        eng.ctl.store(C.F_PS_STOP, 0, 1)
        eng._thread.join(timeout=30)
        eng.ctl.store(C.F_ERROR, 0, 0)
    dist.barrier()
    err, t_err = None, None
    if rank == 1:
        t = time.time()
        try:
            for s in range(40):
                x, y = _data(rank, s % 4)
                opt.zero_grad()
                torch.nn.functional.cross_entropy(m(x), y).backward()
                opt.step()
        except RuntimeError as e:
            err, t_err = str(e), time.time() - t
    dist.barrier()
    try:
        opt.close()
    except Exception:
        pass
    return {"err": err, "t_err": t_err}


def test_worker_raises_when_ps_loop_goes_silent():
    out = run_world(_ps_silent, 2, timeout=180)
    assert out[1]["err"] is not None and "silent" in out[1]["err"], out[1]
    assert out[1]["t_err"] < 15.0


def _open_timeout(rank, world):
    import hipps
    from hipps.parallel.ps_async import IPCOpenTimeout

    m = _mlp()
    t = time.time()
    try:
        hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async")
    except IPCOpenTimeout as e:
        return {"kind": "timeout", "msg": str(e), "t": time.time() - t}
    except RuntimeError as e:
        return {"kind": "runtime", "msg": str(e), "t": time.time() - t}
    return {"kind": "none", "t": time.time() - t}


def test_mailbox_import_timeout_fails_every_rank_fast(monkeypatch):
    """HIPPS_IPC_OPEN_DELAY_S makes every import outlast HIPPS_IPC_OPEN_TIMEOUT_S: rank 1 times out,
    rank 2 does not pile on (its turn never comes), and all three ranks raise IPCOpenTimeout
    together, with the stuck thread's /proc diagnostic in the message."""
    monkeypatch.setenv("HIPPS_IPC_OPEN_DELAY_S", "20")
    monkeypatch.setenv("HIPPS_IPC_OPEN_TIMEOUT_S", "2")
    out = run_world(_open_timeout, 3, timeout=120)
    assert [o["kind"] for o in out] == ["timeout"] * 3, out
    assert "wchan=" in out[0]["msg"] and "rank 1" in out[0]["msg"]
    assert max(o["t"] for o in out) < 15.0


def _mapped(rank, world):
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async", bucket_mb=0.0005)
    eng = opt.engine
    r = {"mapped": eng.mapped_bytes, "ring": eng.ring_bytes, "pub": eng.NPUB * eng.pub_bytes,
         "own": eng.rings[rank] is not None, "others": sum(x is not None for i, x in enumerate(eng.rings) if i != rank)}
    for s in range(3):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    return r


def test_worker_maps_only_its_ring_and_the_publish_region():
    out = run_world(_mapped, 3, timeout=120)
    assert out[0]["others"] == 2  # the PS holds every ring
    for r in (1, 2):
        o = out[r]
        assert o["own"] and o["others"] == 0
        assert o["mapped"] == o["ring"] + o["pub"]


def test_llama8b_w8_default_geometry_fits():
    """Config 5 at W=8, co-located PS, library defaults: the planned geometry fits 90 % of one
    MI355X (288 GB) before activations, by lowering NPUB to 2 and shrinking the rings."""
    from hipps.models import transformer
    from hipps.parallel.ps_async import budget_for_shapes

    with torch.device("meta"):
        model = transformer.build("llama3-8b")
    shapes = [tuple(p.shape) for p in model.parameters()]
    b = budget_for_shapes(shapes, 8)
    assert b["fits"] == 1, b
    assert b["total"] <= 270e9
    assert b["npub"] == 2
    # the ring still holds two of the largest message (the 1 GB embedding bucket)
    big = budget_for_shapes(shapes, 8, hbm_bytes=None)
    assert big["npub"] == 4 and big["total"] > b["total"]


def test_small_models_keep_the_full_geometry():
    from hipps.models import resnet50
    from hipps.parallel.ps_async import budget_for_shapes

    with torch.device("meta"):
        model = resnet50()
    b = budget_for_shapes([tuple(p.shape) for p in model.parameters()], 8)
    assert b["npub"] == 4 and b["fits"] == 1


def _chunked(rank, world, chunk_mb, gran):
    import os

    import hipps

    if chunk_mb:
        os.environ["HIPPS_IPC_CHUNK_MB"] = str(chunk_mb)
    else:
        os.environ.pop("HIPPS_IPC_CHUNK_MB", None)
    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", bucket_mb=0.0005, max_delay=0,
                    accumulate=world, ps_granularity=gran, mailbox_slots=3)
    info = {"npc": opt.engine.npc, "nrc": opt.engine.nrc}
    for s in range(6):
        x, y = _data(0, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    return {"info": info, "params": [p.detach().clone() for p in m.parameters()]}


@pytest.mark.parametrize("gran", ["bucket", "model"])
def test_chunked_mailbox_bitwise(gran):
    """The mailbox as several allocations (publish buffers in 256-aligned chunks, rings whose
    messages never straddle a chunk; what a multi-GB mailbox needs on the GPU) trains bit for bit
    like one allocation per region."""
    a = run_world(_chunked, 2, 0.25, gran, timeout=180)
    b = run_world(_chunked, 2, 0, gran, timeout=180)
    assert a[0]["info"]["npc"] >= 3 and a[0]["info"]["nrc"] >= 2, a[0]["info"]
    assert b[0]["info"] == {"npc": 1, "nrc": 1}
    for r in range(2):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def test_llama8b_w8_adam_fits():
    """Config 5 at W=8 with the reference's Adam (two fp32 moments on the PS, ps.py:217-261):
    rank 0 fits within 85 % of 288 GB -- the M = 1 per-bucket accumulator is one bucket-sized
    scratch (not a model-sized fp32 buffer) and rank 0's worker pushes its buckets straight into
    its ring (no 16 GB wire image)."""
    from hipps.models import transformer
    from hipps.parallel.ps_async import HBM_FRACTION, budget_for_shapes

    with torch.device("meta"):
        model = transformer.build("llama3-8b")
    shapes = [tuple(p.shape) for p in model.parameters()]
    b = budget_for_shapes(shapes, 8, opt_floats=2)
    assert b["fits"] == 1, b
    assert b["total"] <= HBM_FRACTION * 288e9
    assert b["accumulator"] < 3e9 and b["worker_wire"] < 1e6
    # M > 1 (or whole-model versions) needs the full accumulator again
    full = budget_for_shapes(shapes, 8, opt_floats=2, accumulate=4, hbm_bytes=None)
    assert full["accumulator"] >= 4 * sum(math.prod(s) for s in shapes)
