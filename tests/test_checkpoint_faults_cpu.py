"""Checkpoint/resume exactness and async-PS failure handling (fault injection), CPU."""
import os
import time

import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp


def _run(rank, world, mode, steps_a, steps_b, ckpt, codec, max_delay, legacy=None, optim="SGD"):
    import hipps
    from hipps.utils import checkpoint

    def make():
        m = _mlp()
        kw = dict(mode=mode, code=codec)
        if mode == "ps_async":
            kw["max_delay"] = max_delay
            if world > 1:  # every update sums all workers' messages in rank order: deterministic
                kw["accumulate"] = world
        if optim == "Adam":
            return m, hipps.Adam(m.named_parameters(), lr=0.01, **kw)
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
        if legacy is not None and rank == 0:  # rewrite ps.pt in the pre-chunk_steps layout
            path = os.path.join(ckpt, "ps.pt")
            ps = torch.load(path, weights_only=True)
            del ps["chunk_steps"]
            if legacy == "mom_started":
                ps["mom_started"] = [0]
            torch.save(ps, path)
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


@pytest.mark.parametrize("steps_a,steps_b", [(3, 2), (2, 3)])
def test_resume_is_exact_async_default_granularity(tmp_path, steps_a, steps_b):
    """the async PS under the library defaults (ps_granularity='auto' -> per-bucket
    versions, 16 MB buckets, stale_lookahead=0), two workers, odd step counts on either side of
    the checkpoint: the resumed run equals the straight one bit for bit."""
    from hipps.config import PSConfig

    d = PSConfig()
    assert (d.ps_granularity, d.bucket_mb, d.stale_lookahead) == ("auto", 16.0, 0.0)
    straight = run_world(_run, 2, "ps_async", steps_a, steps_b, None, "fp32", 0)
    resumed = run_world(_run, 2, "ps_async", steps_a, steps_b, str(tmp_path / "ck"), "fp32", 0)
    for r in range(2):
        for a, b in zip(straight[r], resumed[r]):
            torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("optim,legacy", [("SGD", "mom_started"), ("SGD", "none"), ("Adam", "none")])
def test_resume_from_checkpoint_without_chunk_steps(tmp_path, optim, legacy):
    """a checkpoint written before per-chunk step counts existed stores only per-group
    counts (SGD: 'mom_started').  Loading it must rebuild the counts, or the first step after the
    resume would restart every momentum buffer (buf = d_p) and Adam's bias correction at t=1."""
    straight = run_world(_run, 1, "local", 3, 3, None, "fp32", 0, None, optim)
    resumed = run_world(_run, 1, "local", 3, 3, str(tmp_path / "ck"), "fp32", 0, legacy, optim)
    for a, b in zip(straight[0], resumed[0]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


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


def _async_ckpt(rank, world, steps_a, steps_b, ckpt, gran="model"):
    """Free-running AsySG-InCon (max_delay=-1) with a slowed PS: the workers' pushes are still
    landing when every rank calls save(); the PS is quiesced between messages for the snapshot."""
    import hipps
    from hipps.utils import checkpoint

    def make():
        m = _mlp()
        return m, hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", max_delay=-1,
                            bucket_mb=0.0005, mailbox_slots=2, ps_granularity=gran)

    m, opt = make()
    for s in range(steps_a):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    nb = len(opt.engine.plan.buckets)
    checkpoint.save(opt, ckpt, m)
    opt.close()
    m, opt = make()
    checkpoint.load(opt, ckpt, m)
    losses = []
    for s in range(steps_a, steps_a + steps_b):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.item())
        opt.step()
    eng = opt.engine
    opt.close()
    return {"stats": eng.ps_stats(), "nb": nb, "losses": losses}


def test_async_checkpoint_quiesce_while_workers_push(tmp_path, monkeypatch):
    """ADVICE r1 / VERDICT r2: W=2, max_delay=-1, whole-model versions (the invariants below are
    the whole-model ones; per-bucket versions: the next test).  The snapshot is one consistent PS state:
    version * M + pending count == messages (steps) accumulated, and the per-worker consumed
    sequence numbers are whole steps or mid-step; after the restore every later step is accounted
    once and the version continues from the snapshot's."""
    monkeypatch.setenv("HIPPS_PS_LOOP_DELAY_US", "4000")
    ck = str(tmp_path / "ck")
    out = run_world(_async_ckpt, 2, 5, 6, ck, timeout=240)
    ps = torch.load(os.path.join(ck, "ps.pt"), weights_only=True)
    M = 2
    assert ps["version"] * M + ps["acc_count"] == ps["ps_accumulated"], ps
    nb = out[0]["nb"]
    assert nb >= 3
    # the snapshot was taken while pushes were still in flight: not everything pushed was consumed
    assert sum(ps["ps_seen"]) <= 2 * 5 * nb
    st = out[0]["stats"]
    assert st["accumulated"] == 2 * 6  # every post-restore step of both workers, exactly once
    assert st["version"] == ps["version"] + (ps["acc_count"] + 2 * 6) // M
    for r in range(2):
        assert all(l == l for l in out[r]["losses"])  # finite


def test_async_checkpoint_quiesce_bucket_versions(tmp_path, monkeypatch):
    """The same under per-bucket versions (ps_granularity='bucket', the 'auto' choice on the ipc
    transport): the snapshot is taken between messages, so every bucket has consumed all
    accumulated steps plus at most one per worker (the message of that worker's step in progress
    arrived before the step's last bucket): accumulated <= ver_b * M + count_b <= accumulated + W, the global version is the
    slowest bucket's, and after the restore every later step is accounted once."""
    monkeypatch.setenv("HIPPS_PS_LOOP_DELAY_US", "4000")
    ck = str(tmp_path / "ck")
    out = run_world(_async_ckpt, 2, 5, 6, ck, "bucket", timeout=240)
    ps = torch.load(os.path.join(ck, "ps.pt"), weights_only=True)
    M = 2
    acc = ps["ps_accumulated"]
    es = torch.load(os.path.join(ck, "rank0.pt"), weights_only=True)["engine"]  # per-bucket PS words
    per_bucket = [v * M + c for v, c in zip(es["ver_b"], es["acc_count_b"])]
    # each of the W=2 workers may have one step in progress whose message for bucket b was consumed
    assert all(acc <= n <= acc + 2 for n in per_bucket), (acc, per_bucket)
    assert ps["version"] == min(es["ver_b"])
    st = out[0]["stats"]
    assert st["accumulated"] == 2 * 6
    for r in range(2):
        assert all(l == l for l in out[r]["losses"])
