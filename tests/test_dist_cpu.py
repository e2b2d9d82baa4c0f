"""Multi-process (gloo, CPU) tests of the exchange engines.

BASELINE config 1: 2-layer MLP (784-200-10, MNIST-shaped synthetic data), sync PS, CPU,
world_size 2.  Replaces the reference's `mpirun -n 2 py.test` (Makefile:3).
"""
import pytest
import torch

from dist_util import run_world


def _mlp():
    from hipps.models.mlp import mlp_mnist

    torch.manual_seed(0)
    return mlp_mnist()


def _data(rank, step):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(32, 784, generator=g), torch.randint(0, 10, (32,), generator=g)


def _train(rank, world, mode, codec, steps, opt_name):
    import hipps

    m = _mlp()
    cls = hipps.SGD if opt_name == "sgd" else hipps.Adam
    kw = dict(lr=0.05, momentum=0.9) if opt_name == "sgd" else dict(lr=1e-3)
    opt = cls(m.named_parameters(), m.parameters(), mode=mode, code=codec, **kw)
    for s in range(steps):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        loss, data = opt.step()
    opt.close()
    return [p.detach().clone() for p in m.parameters()], data


def _simulate(world, steps, opt_name):
    """Single process: gradient = sum over ranks (ps.py:176) applied with the same optimizer."""
    import hipps

    m = _mlp()
    ms = [_mlp() for _ in range(world)]
    cls = hipps.SGD if opt_name == "sgd" else hipps.Adam
    kw = dict(lr=0.05, momentum=0.9) if opt_name == "sgd" else dict(lr=1e-3)
    opt = cls(m.named_parameters(), m.parameters(), mode="local", **kw)
    for s in range(steps):
        gsum = None
        for r in range(world):
            ms[r].load_state_dict(m.state_dict())
            ms[r].zero_grad()
            x, y = _data(r, s)
            torch.nn.functional.cross_entropy(ms[r](x), y).backward()
            g = [p.grad.clone() for p in ms[r].parameters()]
            gsum = g if gsum is None else [a + b for a, b in zip(gsum, g)]
        opt.zero_grad()
        for p, g in zip(m.parameters(), gsum):
            p.grad = g.clone()
        opt.step()
    return [p.detach().clone() for p in m.parameters()]


@pytest.mark.parametrize("mode", ["allgather", "ps_sync"])
@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_sync_modes_match_single_process_sum(mode, opt_name):
    out = run_world(_train, 2, mode, "fp32", 4, opt_name)
    p0, p1 = out[0][0], out[1][0]
    for a, b in zip(p0, p1):
        assert torch.equal(a, b), "replicas diverged"
    want = _simulate(2, 4, opt_name)
    for a, b in zip(p0, want):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    assert out[0][1]["grad_bytes_sent"] > 0


@pytest.mark.parametrize("codec", ["bf16", "int8", "topk:0.05", "topk_int8:0.05", "threshold:0.01:0.2"])
def test_allgather_codecs_keep_replicas_identical(codec):
    out = run_world(_train, 2, "allgather", codec, 3, "sgd")
    for a, b in zip(out[0][0], out[1][0]):
        assert torch.equal(a, b)


def _ps_sync_bf16(rank, world):
    import hipps

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="ps_sync", code="topk:0.1", param_wire="bf16")
    for s in range(3):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    return [p.detach().clone() for p in m.parameters()]


def test_ps_sync_three_ranks_bf16_params():
    out = run_world(_ps_sync_bf16, 3)
    for r in (1, 2):
        for a, b in zip(out[0], out[r]):
            torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2)
