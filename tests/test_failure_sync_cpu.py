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


_WD_SCRIPT = r"""
import sys, time
sys.path.insert(0, {root!r})
from hipps.parallel.watchdog import CommWatchdog

class Ev:
    def __init__(self, done): self.done = done
    def query(self): return self.done

aborted = []
wd = CommWatchdog(0.01, rank=0, on_abort=lambda: print("ABORT", flush=True))
kind = sys.argv[1]
wd.watch(Ev(True), "finished collective")
if kind == "hang":
    wd.watch(Ev(False), "allgather step 3 collectives")
elif kind == "error":
    def poll():
        raise RuntimeError("RCCL communicator failed: remote process exited")
    wd.watch(Ev(False), "ps_sync step 2 bcast", poll)
time.sleep(9)
print("pending", wd.pending(), flush=True)
"""


@pytest.mark.parametrize("kind", ["ok", "hang", "error"])
def test_watchdog_follows_enqueued_device_exchanges(kind, tmp_path):
    """transport='rccl' exchanges return once enqueued; the watchdog keeps following
    their completion event -- a collective that never completes, or an asynchronous RCCL error,
    aborts the communicator and exits with status 3 instead of surfacing later in user code."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "wd.py"
    f.write_text(_WD_SCRIPT.format(root=root))
    r = subprocess.run([sys.executable, str(f), kind], capture_output=True, text=True, timeout=60)
    if kind == "ok":
        assert r.returncode == 0 and "pending 0" in r.stdout, r.stderr
    else:
        assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
        assert "ABORT" in r.stdout
        assert ("did not complete" in r.stderr) if kind == "hang" else ("failed asynchronously" in r.stderr)
