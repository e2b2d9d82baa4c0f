"""Parameter-set semantics (reference ps.py:118-119, 150-153, 178-179) and gradient accumulation.

* frozen parameters (requires_grad=False) are not hooked, exchanged or updated;
* a parameter that produced no gradient this step is skipped -- no weight decay, no momentum
  step -- like the reference's ``if p.grad is None: continue``; the sync modes OR the ranks'
  presence so replicas stay identical, the async PS ORs the accumulated messages';
* ``require_all_grads=True`` restores the reference's ValueError (ps.py:118-119);
* two backward() calls before step() equal one backward() of the summed loss, with or without
  ``opt.no_sync()``.
"""
import pytest
import torch
import torch.nn as nn

from dist_util import run_world


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = nn.Linear(16, 16)
        self.b = nn.Linear(16, 4)
        self.unused = nn.Linear(16, 16)  # never called in forward
        self.frozen = nn.Linear(16, 16)
        self.frozen.requires_grad_(False)

    def forward(self, x):
        return self.b(torch.relu(self.a(x) + self.frozen(x)))


def _data(rank, step):
    g = torch.Generator().manual_seed(100 * step + rank)
    return torch.randn(8, 16, generator=g), torch.randint(0, 4, (8,), generator=g)


def _train(rank, world, mode, steps=3, transport="ipc"):
    import hipps

    m = Net()
    keep = {n: p.detach().clone() for n, p in m.named_parameters() if n.startswith(("unused", "frozen"))}
    opt = hipps.SGD(m.named_parameters(), lr=0.1, momentum=0.9, weight_decay=0.1, mode=mode, max_delay=0,
                    accumulate=world, async_transport=transport)
    for s in range(steps):
        x, y = _data(rank, s)
        opt.zero_grad()
        nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    after = {n: p.detach().clone() for n, p in m.named_parameters()}
    moved = not torch.equal(after["a.weight"], Net().a.weight.detach())
    return {"keep": keep, "after": after, "moved": moved}


@pytest.mark.parametrize("mode,world,transport", [("local", 1, "ipc"), ("allgather", 2, "ipc"), ("ps_sync", 2, "ipc"),
                                                   ("ps_async", 2, "ipc"), ("ps_async", 2, "p2p")])
def test_frozen_and_unused_params_untouched(mode, world, transport):
    out = run_world(_train, world, mode, 3, transport)
    for r in range(world):
        o = out[r]
        assert o["moved"], "trained parameters must move"
        for n, v in o["keep"].items():
            assert torch.equal(o["after"][n], v), f"{mode}: {n} changed (rank {r})"


def _strict(rank, world):
    import hipps

    m = Net()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, mode="local", require_all_grads=True)
    x, y = _data(0, 0)
    nn.functional.cross_entropy(m(x), y).backward()
    try:
        opt.step()
    except ValueError as e:
        return str(e)
    return None


def test_require_all_grads_raises_like_reference():
    msg = run_world(_strict, 1)[0]
    assert msg is not None and "unused.weight" in msg


def test_duplicate_names_rejected():
    import hipps

    p, q = nn.Parameter(torch.zeros(3)), nn.Parameter(torch.zeros(3))
    with pytest.raises(ValueError, match="names not unique"):
        hipps.SGD([("w", p), ("w", q)], lr=0.1, mode="local")


def test_zero_grad_set_to_none_false_counts_as_present():
    """torch semantics: zero-filled grads are grads -> weight decay still applies."""
    import hipps

    m = Net()
    w0 = m.unused.weight.detach().clone()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, weight_decay=0.1, mode="local")
    x, y = _data(0, 0)
    opt.zero_grad(set_to_none=False)
    nn.functional.cross_entropy(m(x), y).backward()
    opt.step()
    opt.close()
    torch.testing.assert_close(m.unused.weight.detach(), w0 * (1 - 0.1 * 0.1))


def _mlp():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(16, 16), nn.ReLU(), nn.Linear(16, 4))


def _accum(rank, world, mode, how, codec="fp32", net="net"):
    import hipps

    m = Net() if net == "net" else _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, momentum=0.9, mode=mode, code=codec)
    for s in range(2):
        x, y = _data(rank, s)
        opt.zero_grad()
        if how == "once":
            (nn.functional.cross_entropy(m(x[:4]), y[:4]) + nn.functional.cross_entropy(m(x[4:]), y[4:])).backward()
        elif how == "twice":
            nn.functional.cross_entropy(m(x[:4]), y[:4]).backward()
            nn.functional.cross_entropy(m(x[4:]), y[4:]).backward()
        else:
            with opt.no_sync():
                nn.functional.cross_entropy(m(x[:4]), y[:4]).backward()
            nn.functional.cross_entropy(m(x[4:]), y[4:]).backward()
        opt.step()
    opt.close()
    return [p.detach().clone() for p in m.parameters()]


@pytest.mark.parametrize("mode,world", [("local", 1), ("allgather", 2)])
@pytest.mark.parametrize("how", ["twice", "no_sync"])
@pytest.mark.parametrize("net", ["net", "mlp"])  # mlp: every bucket is encoded during the 1st backward
def test_gradient_accumulation_equals_summed_loss(mode, world, how, net):
    want = run_world(_accum, world, mode, "once", "fp32", net)
    got = run_world(_accum, world, mode, how, "fp32", net)
    for r in range(world):
        for a, b in zip(got[r], want[r]):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)


def _accum_ef(rank, world):
    try:
        _accum(rank, world, "local", "twice", codec="topk:0.5", net="mlp")
    except RuntimeError as e:
        return str(e)
    return None


def test_accumulation_with_error_feedback_codec_needs_no_sync():
    msg = run_world(_accum_ef, 1)[0]
    assert msg is not None and "no_sync" in msg


def _metrics(rank, world, mode):
    import hipps

    m = Net()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, mode=mode, code="bf16")
    x, y = _data(rank, 0)
    nn.functional.cross_entropy(m(x), y).backward()
    _, data = opt.step()
    opt.close()
    return data


@pytest.mark.parametrize("mode,world", [("local", 1), ("allgather", 2), ("ps_sync", 2), ("ps_async", 2)])
def test_step_metrics_keep_reference_keys(mode, world):
    data = run_world(_metrics, world, mode)[0]
    for k in ("comm_wait", "optim_step_time", "decode_time", "msg_bytes", "packaged_bytes", "code_wait",
              "iallgather_prepare_time", "isend_time", "grad_bytes_sent"):
        assert k in data, (mode, k)
    assert data["msg_bytes"] > 0 and data["packaged_bytes"] >= data["msg_bytes"]


def test_mpi_ps_factory_and_reference_constructor():
    """``MPI_PS(named_params, *params, names=, optim=, code=, use_mpi=, cuda=, **torch_kwargs)``
    (ps.py:54-59) builds the subclass its ``optim`` names and keeps the reference attributes."""
    import hipps

    m = torch.nn.Linear(4, 2)
    o = hipps.MPI_PS(m.named_parameters(), m.parameters(), names=["w", "b"], optim="sgd", code=None, use_mpi=True,
                     cuda=False, lr=0.1, momentum=0.9)
    assert isinstance(o, hipps.SGD) and o.optim == "sgd" and o.use_mpi and o.cuda is False and o.names == ["w", "b"]
    o.zero_grad()
    m(torch.randn(3, 4)).sum().backward()
    loss, data = o.step()
    assert loss is None and {"msg_bytes", "packaged_bytes", "iallgather_prepare_time"} <= set(data)
    o.close()
    a = hipps.MPI_PS(m.named_parameters(), optim="adam", lr=1e-3)
    assert isinstance(a, hipps.Adam)
    a.close()
    with pytest.raises(ValueError):
        hipps.MPI_PS(m.named_parameters(), optim="rmsprop", lr=0.1)
    with pytest.raises(ValueError):
        hipps.SGD(m.named_parameters(), optim="adam", lr=0.1)
