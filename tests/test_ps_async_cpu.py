"""Async PS (AsySG-InCon) protocol tests on CPU: shm control block + shm mailboxes, gloo rendezvous."""
import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp


def _train_async(rank, world, steps, codec, accumulate, max_delay, staleness, opt_name="sgd", bucket_mb=64.0,
                 slots=0, transport="ipc", main_collectives=False):
    import hipps

    m = _mlp()
    if rank:  # deliberately different init: the PS's version 0 must win
        torch.manual_seed(100 + rank)
        for p in m.parameters():
            p.data.normal_()
    cls = hipps.SGD if opt_name == "sgd" else hipps.Adam
    kw = dict(lr=0.05, momentum=0.9) if opt_name == "sgd" else dict(lr=1e-3)
    opt = cls(m.named_parameters(), mode="ps_async", code=codec, accumulate=accumulate, max_delay=max_delay,
              staleness=staleness, bucket_mb=bucket_mb, mailbox_slots=slots, async_transport=transport, **kw)
    nb = len(opt.engine.plan.buckets)
    init = [p.detach().clone() for p in m.parameters()]
    losses = []
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.item())
        opt.step()
        if main_collectives:  # rank 0's main thread uses the default group while its PS thread serves
            import torch.distributed as dist

            t = torch.ones(1)
            dist.all_reduce(t)
            assert t.item() == world
            dist.barrier()
    eng = opt.engine
    opt.close()  # drains: the PS thread exits only after consuming every pushed message
    stats = eng.ps_stats()
    master = eng.final_params() if rank == 0 else None
    return {"init": init, "losses": losses, "stats": stats, "master": master, "nb": nb,
            "params": [p.detach().clone() for p in m.parameters()]}


@pytest.mark.parametrize("bucket_mb,slots", [(64.0, 0), (0.0005, 2), (0.0005, 1)])
def test_async_single_rank_sync_delay_equals_local(bucket_mb, slots):
    """W=1, M=1, max_delay=0: every step waits for its own update -> identical to local SGD, also
    when each step is streamed as several bucket messages through a 1- or 2-slot mailbox."""
    import hipps

    out = run_world(_train_async, 1, 5, "fp32", 1, 0, -1, "sgd", bucket_mb, slots)
    if bucket_mb < 1:
        assert out[0]["nb"] >= 3
    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="local")
    for s in range(5):
        x, y = _data(0, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    for a, b in zip(out[0]["params"], m.parameters()):
        torch.testing.assert_close(a, b.detach(), rtol=0, atol=0)
    assert out[0]["stats"]["updates"] == 5


@pytest.mark.parametrize("codec,bucket_mb", [("fp32", 64.0), ("bf16", 0.0005), ("topk_int8:0.1", 0.0005),
                                            ("threshold:0.001:0.3", 0.0005)])
def test_async_three_ranks_converges_and_accounts(codec, bucket_mb):
    steps = 12
    out = run_world(_train_async, 3, steps, codec, 0, -1, -1, "sgd", bucket_mb, 0)
    st = out[0]["stats"]
    # every pushed message is accumulated exactly once; M = W = 3
    assert st["accumulated"] == 3 * steps
    assert st["updates"] == steps
    # all replicas adopted the PS's version 0 at start
    for r in (1, 2):
        for a, b in zip(out[0]["init"], out[r]["init"]):
            assert torch.equal(a, b)
    # training made progress on every worker
    for r in range(3):
        L = out[r]["losses"]
        assert sum(L[-4:]) / 4 < sum(L[:4]) / 4
    # after close the PS master holds the last version; bounded staleness
    assert st["staleness_sum"] / st["accumulated"] < 4


def test_async_max_delay_zero_three_ranks_is_ssp_synchronous():
    out = run_world(_train_async, 3, 6, "fp32", 3, 0, -1)
    st = out[0]["stats"]
    assert st["updates"] == 6 and st["accumulated"] == 18


def test_async_staleness_drop_and_adam():
    # M=1 with 3 workers: versions advance on every message; staleness=0 drops most laggards
    out = run_world(_train_async, 3, 6, "fp32", 1, -1, 0, "adam")
    st = out[0]["stats"]
    assert st["accumulated"] + st["drops"] == 18
    assert st["updates"] == st["accumulated"]


@pytest.mark.parametrize("codec,bucket_mb,slots", [("fp32", 64.0, 0), ("bf16", 0.0005, 2), ("topk_int8:0.1", 0.0005, 0)])
def test_async_p2p_transport_converges_and_accounts(codec, bucket_mb, slots):
    """Two-sided send/recv transport (pair channels; RCCL on GPU, gloo here): same protocol,
    same accounting as the one-sided mailbox."""
    steps = 10
    out = run_world(_train_async, 3, steps, codec, 0, -1, -1, "sgd", bucket_mb, slots, "p2p")
    st = out[0]["stats"]
    assert st["accumulated"] == 3 * steps and st["updates"] == steps
    for r in (1, 2):
        for a, b in zip(out[0]["init"], out[r]["init"]):
            assert torch.equal(a, b)
    for r in range(3):
        L = out[r]["losses"]
        assert sum(L[-3:]) / 3 < sum(L[:3]) / 3


def test_async_p2p_max_delay_zero_matches_ipc():
    """SSP bound 0 with M = W: both transports apply the same synchronous update sequence."""
    a = run_world(_train_async, 2, 5, "fp32", 2, 0, -1, "sgd", 64.0, 0, "p2p")
    b = run_world(_train_async, 2, 5, "fp32", 2, 0, -1, "sgd", 64.0, 0, "ipc")
    for r in range(2):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def _ipc_fails_then_p2p(rank, world):
    """Rank 1 cannot map the PS mailbox: every rank must raise together (nobody left in a barrier),
    the failed engine must leave no hooks behind, and the same async PS then trains over 'p2p' --
    the recovery bench.py performs at N > 1."""
    import hipps
    from hipps.ops import _native

    C = _native.native()
    m = _mlp()
    if rank == 1:
        real = C.HostMailbox

        class Refuse:
            def __init__(self, name, total, create):
                if not create:
                    raise OSError("simulated: mailbox mapping refused")
                self._m = real(name, total, create)

        C.HostMailbox = Refuse
    err = None
    try:
        hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="fp32")
    except RuntimeError as e:
        err = str(e)
    finally:
        if rank == 1:
            C.HostMailbox = real
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="fp32",
                    async_transport="p2p")
    for s in range(3):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    eng = opt.engine
    opt.close()
    return {"err": err, "stats": eng.ps_stats() if rank == 0 else None}


def test_ipc_mapping_failure_is_collective_and_p2p_recovers():
    out = run_world(_ipc_fails_then_p2p, 2)
    assert all(o["err"] and "mapping the PS mailbox failed" in o["err"] and "rank 1" in o["err"] for o in out), out
    assert out[0]["stats"]["accumulated"] == 2 * 3


def test_async_p2p_slow_ps_with_main_thread_collectives(monkeypatch):
    """with a slowed PS loop the PS sees a worker's parameter request and its next
    step's announcement in one iteration; parameters travel on their own process group and the
    request is answered first, so the pair channel cannot deadlock.  Rank 0's main thread runs
    all_reduce + barrier on the default group every step meanwhile."""
    monkeypatch.setenv("HIPPS_PS_LOOP_DELAY_US", "3000")
    steps = 8
    out = run_world(_train_async, 3, steps, "fp32", 0, -1, -1, "sgd", 0.0005, 2, "p2p", True)
    st = out[0]["stats"]
    assert st["accumulated"] == 3 * steps and st["updates"] == steps


def _dedicated(rank, world, steps, transport):
    """The reference's topology (README.md:64-75): rank 0 only serves, ranks 1..W-1 train."""
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", ps_dedicated=True,
                    async_transport=transport)
    if rank == 0:
        assert opt.ps_only
        with pytest.raises(RuntimeError, match="dedicated"):
            opt.step()
        st = opt.serve(timeout_s=120)
        return {"stats": st, "losses": []}
    assert not opt.ps_only
    losses, stale = [], []
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.item())
        _, data = opt.step()
        stale.append(data["staleness"])
    info = opt.engine.transport_info()
    opt.close()
    return {"losses": losses, "info": info, "stale": stale}


@pytest.mark.parametrize("transport", ["ipc", "p2p"])
def test_async_dedicated_ps_topology(transport):
    steps = 8
    out = run_world(_dedicated, 3, steps, transport)
    st = out[0]["stats"]
    # M defaults to the number of workers (2): one update per round of worker steps
    assert st["accumulated"] == 2 * steps and st["updates"] == steps, st
    for r in (1, 2):
        assert out[r]["info"]["ps_dedicated"] and out[r]["info"]["accumulate"] == 2
        assert sum(out[r]["losses"][-3:]) < sum(out[r]["losses"][:3])
        assert all(s >= 0 for s in out[r]["stale"])


def _bucketwise(rank, world, steps, max_delay):
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", ps_granularity="bucket",
                    bucket_mb=0.0005, max_delay=max_delay, accumulate=world)
    nb = len(opt.engine.plan.buckets)
    losses = []
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.item())
        opt.step()
    eng = opt.engine
    lver = list(eng._lver_b)
    opt.close()
    return {"stats": eng.ps_stats(), "nb": nb, "losses": losses, "lver_b": lver,
            "params": [p.detach().clone() for p in m.parameters()]}


def test_async_bucket_granularity_trains_and_accounts():
    """ps_granularity='bucket' (README.md:64-76): per-bucket PS updates and per-bucket publication,
    3 ranks over the shm mailbox; every message accounted, global version = rounds, loss falls."""
    steps = 10
    out = run_world(_bucketwise, 3, steps, -1)
    st = out[0]["stats"]
    nb = out[0]["nb"]
    assert nb >= 3
    assert st["accumulated"] == 3 * steps and st["version"] == steps and st["updates"] == steps
    assert st["bucket_updates"] == steps * nb
    for r in range(3):
        L = out[r]["losses"]
        assert sum(L[-3:]) < sum(L[:3])


def test_async_bucket_granularity_max_delay_zero_matches_model():
    """With max_delay=0 and M = W every bucket's update sequence is the synchronous one: bucket
    granularity gives the same parameters as whole-model granularity."""
    a = run_world(_bucketwise, 2, 5, 0)
    b = run_world(_train_async, 2, 5, "fp32", 2, 0, -1, "sgd", 0.0005, 0, "ipc")
    for r in range(2):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def _early(rank, world, steps, push_early, granularity="model", twice=False):
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", bucket_mb=0.0005,
                    max_delay=0, accumulate=world, push_early=push_early, ps_granularity=granularity)
    nb = len(opt.engine.plan.buckets)
    early = []
    err = None
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        if twice:
            torch.nn.functional.cross_entropy(m(x), y).backward()
        try:
            _, data = opt.step()
        except RuntimeError as e:
            err = str(e)
            break
        early.append(data["pushed_early"])
    err2 = None
    if err is not None:  # a caller that catches the error and keeps training
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        try:
            opt.step()
        except RuntimeError as e:
            err2 = str(e)
    opt.close()
    return {"nb": nb, "early": early, "err": err, "err2": err2,
            "params": [p.detach().clone() for p in m.parameters()]}


@pytest.mark.parametrize("granularity", ["model", "bucket"])
def test_async_push_early_during_backward_matches_push_at_step(granularity):
    """push_early: every bucket's message leaves from its backward hook (all nb of them: every
    parameter gets a gradient), and with max_delay=0 the parameters are bit-identical to pushing
    everything at step()."""
    a = run_world(_early, 2, 5, "on", granularity)
    b = run_world(_early, 2, 5, "off", granularity)
    for r in range(2):
        assert a[r]["nb"] >= 3 and all(e == a[r]["nb"] for e in a[r]["early"]), a[r]["early"]
        assert all(e == 0 for e in b[r]["early"])
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def test_async_push_early_rejects_a_late_gradient():
    """A second backward() before step() adds gradient to buckets already pushed: an error, not a
    silently dropped gradient (opt.no_sync() or push_early='off' are the ways out)."""
    out = run_world(_early, 1, 2, "on", "model", True)
    assert out[0]["err"] is not None and "no_sync" in out[0]["err"]
    # the early messages already moved the worker's sequence, so the engine must not
    # accept another step (later messages would land on the wrong buckets of the PS)
    assert out[0]["err2"] is not None and "cannot continue" in out[0]["err2"]


def _gran(rank, world, transport):
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", bucket_mb=0.0005,
                    ps_granularity="auto", async_transport=transport, max_delay=0)
    info = dict(opt.engine.transport_info())
    x, y = _data(rank, 0)
    opt.zero_grad()
    torch.nn.functional.cross_entropy(m(x), y).backward()
    opt.step()
    opt.close()
    return info


def test_async_granularity_auto():
    """ps_granularity='auto': per-bucket versions on the ipc transport, whole-model on p2p."""
    assert run_world(_gran, 2, "ipc")[0]["granularity"] == "bucket"
    assert run_world(_gran, 2, "p2p")[0]["granularity"] == "model"


class _HeadPlusUnused(torch.nn.Module):
    """An MLP whose unused layer sits between two used ones in registration order (BERT's pooler
    under an MLM-only loss): its bucket comes early in the ready order."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.fc1 = torch.nn.Linear(784, 64)
        self.unused = torch.nn.Linear(64, 64)
        self.fc2 = torch.nn.Linear(64, 10)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


def _early_unused(rank, world, steps, push_early, granularity):
    import hipps

    m = _HeadPlusUnused()
    w0 = m.unused.weight.detach().clone()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", bucket_mb=0.0005,
                    max_delay=0, accumulate=world, push_early=push_early, ps_granularity=granularity)
    nb = len(opt.engine.plan.buckets)
    unused = {id(m.unused.weight), id(m.unused.bias)}
    n_inc = sum(any(id(opt.store.slots[j].param) in unused for j in b.slot_ids) for b in opt.engine.plan.buckets)
    early = []
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        _, data = opt.step()
        early.append(data["pushed_early"])
    opt.close()
    return {"nb": nb, "n_inc": n_inc, "early": early, "unused_same": torch.equal(m.unused.weight.detach(), w0),
            "params": [p.detach().clone() for p in m.parameters()]}


@pytest.mark.parametrize("granularity", ["model", "bucket"])
def test_async_push_early_past_a_bucket_without_gradients(granularity):
    """A bucket holding a parameter with no gradient (skipped, as ps.py:178-179 skips grad None)
    no longer holds back the buckets behind it in message order: every complete bucket leaves from
    its backward hook, the incomplete one at step() with its presence mask -- and the parameters
    are bit-identical to pushing everything at step(); the unused layer never moves."""
    a = run_world(_early_unused, 2, 4, "on", granularity)
    b = run_world(_early_unused, 2, 4, "off", granularity)
    for r in range(2):
        nb = a[r]["nb"]
        assert nb >= 3
        # every bucket but the ones holding the unused layer (which sit early in the ready order)
        assert 0 < a[r]["n_inc"] < nb - 1
        assert all(e == nb - a[r]["n_inc"] for e in a[r]["early"]), (a[r]["early"], nb, a[r]["n_inc"])
        assert all(e == 0 for e in b[r]["early"])
        assert a[r]["unused_same"] and b[r]["unused_same"]
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def _ring(rank, world, mailbox_mb, granularity):
    import hipps

    m = _HeadPlusUnused()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", bucket_mb=0.0005,
                    max_delay=0, accumulate=world, ps_granularity=granularity, mailbox_mb=mailbox_mb)
    eng = opt.engine
    geo = (eng.SLOTS, eng.ring_bytes, max(eng.msg_ext), sum(eng.msg_ext))
    for s in range(5):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    return {"geo": geo, "params": [p.detach().clone() for p in m.parameters()]}


@pytest.mark.parametrize("granularity,world", [("model", 2), ("bucket", 2), ("bucket", 3)])
def test_async_mailbox_ring_wraps(granularity, world):
    """The per-worker mailbox is a byte ring of variable-size messages (their offsets ride in the
    flag word): a ring of two largest messages, which wraps within every two steps, trains like a
    ring holding two whole steps (bit for bit with two workers)."""
    small = run_world(_ring, world, 1e-6, granularity)
    big = run_world(_ring, world, 4096.0, granularity)
    K, ring, mx, tot = small[0]["geo"]
    assert ring == 2 * (mx + 256) < 2 * tot <= big[0]["geo"][1]
    # two workers' sums are exact in any order; three arrive in any order, so fp32 summation order
    tol = 0 if world == 2 else 1e-6
    for r in range(world):
        for x, y in zip(small[r]["params"], big[r]["params"]):
            torch.testing.assert_close(x, y, rtol=tol, atol=tol)
