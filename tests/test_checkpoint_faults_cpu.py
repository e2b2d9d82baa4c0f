"""Checkpoint/resume exactness and async-PS failure handling (fault injection), CPU."""
import os
import time

import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp


def _run(rank, world, mode, steps_a, steps_b, ckpt, codec, max_delay):
    import hipps
    from hipps.utils import checkpoint

    def make():
        m = _mlp()
        kw = dict(mode=mode, code=codec)
        if mode == "ps_async":
            kw["max_delay"] = max_delay
        return m, hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, **kw)

    m, opt = make()
    for s in range(steps_a):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    if ckpt:
        checkpoint.save(opt, ckpt, m)
        opt.close()
        m, opt = make()  # fresh process state: different init is overwritten by the load
        checkpoint.load(opt, ckpt, m)
    for s in range(steps_a, steps_a + steps_b):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    if mode == "ps_async":
        opt.irequest_params(block_for=opt.engine.ctl.load(opt.engine.C.F_PUB_VER, 0))
    opt.close()
    return [p.detach().clone() for p in m.parameters()]


@pytest.mark.parametrize("mode,W,codec,max_delay", [("allgather", 2, "topk:0.1", 0), ("ps_async", 1, "int8", 0),
                                                    ("ps_sync", 2, "fp32", 0)])
def test_resume_is_exact(tmp_path, mode, W, codec, max_delay):
    straight = run_world(_run, W, mode, 3, 3, None, codec, max_delay)
    resumed = run_world(_run, W, mode, 3, 3, str(tmp_path / "ck"), codec, max_delay)
    for a, b in zip(straight[0], resumed[0]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    assert os.path.exists(tmp_path / "ck" / "ps.pt")
    sd = torch.load(tmp_path / "ck" / "ps.pt", weights_only=True)
    assert sd["mode"] == mode


def _faulty(rank, world, steps):
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_async", dead_after_s=2.0)
    t0 = time.time()
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    eng = opt.engine
    if rank == 0:
        time.sleep(2.5)  # let the dead worker's heartbeat age past dead_after_s
    opt.close()
    return {"stats": eng.ps_stats(), "dead": eng.dead_workers() if rank == 0 else [], "t": time.time() - t0}


def test_async_survives_dead_worker(monkeypatch):
    monkeypatch.setenv("HIPPS_FAULT", "2:3:die")
    out = run_world(_faulty, 3, 8, timeout=120)
    st = out[0]["stats"]
    # ranks 0,1 pushed 8 each; rank 2 pushed 2 before dying -> 18 messages accumulated
    assert st["accumulated"] == 18
    assert st["updates"] == 18 // 3
    assert out[0]["dead"] == [2]


def test_async_slow_worker_and_drop(monkeypatch):
    monkeypatch.setenv("HIPPS_FAULT", "1:1:slow:30,2:2:drop")
    out = run_world(_faulty, 3, 6, timeout=120)
    st = out[0]["stats"]
    assert st["accumulated"] == 6 + 6 + 5
