"""Failure handling in the synchronous modes.

A rank that stops participating (HIPPS_FAULT='1:3:hang') must not stall the others for the
default 10 minutes: the engines' process group times out after ``comm_timeout_s`` (gloo raises;
RCCL aborts the communicator), so rank 0 gets an error within the bound.  A rank that dies
outright (``die``) is detected even faster (the transport sees the peer go away)."""
import os
import time

import pytest
import torch
import torch.multiprocessing as mp

from dist_util import free_port


def _rank(rank, world, port, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import hipps
    from hipps.parallel import dist as hdist
    from test_dist_cpu import _data, _mlp

    hdist.init_from_env(backend="gloo")
    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode=mode, comm_timeout_s=4.0)
    t0 = None
    try:
        for s in range(6):
            x, y = _data(rank, s)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            t0 = time.time()
            opt.step()
        q.put((rank, "finished", 0.0))
    except Exception as e:  # the timeout / peer-loss error
        q.put((rank, type(e).__name__ + ": " + str(e)[:200], time.time() - t0))


@pytest.mark.parametrize("mode", ["allgather", "ps_sync"])
@pytest.mark.parametrize("kind", ["hang", "die"])
def test_dead_peer_fails_fast(monkeypatch, mode, kind):
    monkeypatch.setenv("HIPPS_FAULT", f"1:3:{kind}")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        rank, status, waited = q.get(timeout=120)
        assert rank == 0, status
        assert status != "finished", "rank 0 cannot finish with a dead peer"
        assert waited < 30, f"rank 0 waited {waited:.1f}s for a dead peer ({status})"
    finally:
        for p in ps:
            p.join(timeout=2)
            if p.is_alive():
                p.kill()
                p.join()
