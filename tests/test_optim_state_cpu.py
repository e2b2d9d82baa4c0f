"""Per-parameter optimizer state under skipped gradients (reference ps.py:178-179,
202-205, 241).

The reference keeps optimizer state per parameter: the momentum buffer is created on the
parameter's own first gradient (``buf = d_p``, ps.py:203-205) and Adam's ``state['step']`` only
advances when the parameter has a gradient (ps.py:241), because parameters without one are
skipped (ps.py:178-179).  hipps keeps one int32 update count per 16-element chunk on the device
(``MPI_PS.chunk_steps``) that the fused kernels read and advance under the chunk mask; these tests
pin that against literal per-parameter transcriptions, in one process and in the multi-rank sync
modes (whose presence mask is always built, every rank ORing the others' presence bytes).
"""
import math

import pytest
import torch

from dist_util import run_world


class RefOpt:
    """Per-parameter transcription of ps.py SGD.optim_step / Adam.optim_step with the
    ``if p.grad is None: continue`` skip."""

    def __init__(self, params, kind, lr, momentum=0.0, dampening=0.0, wd=0.0, betas=(0.9, 0.999), eps=1e-8):
        self.params, self.kind = list(params), kind
        self.lr, self.mom, self.damp, self.wd, self.betas, self.eps = lr, momentum, dampening, wd, betas, eps
        self.state = [dict() for _ in self.params]

    @torch.no_grad()
    def step(self):
        for p, st in zip(self.params, self.state):
            if p.grad is None:
                continue
            d_p = p.grad.clone()
            if self.kind == "sgd":
                if self.wd:
                    d_p.add_(p, alpha=self.wd)
                if self.mom:
                    if "momentum_buffer" not in st:
                        buf = st["momentum_buffer"] = torch.zeros_like(p)
                        buf.mul_(self.mom).add_(d_p)
                    else:
                        buf = st["momentum_buffer"]
                        buf.mul_(self.mom).add_(d_p, alpha=1 - self.damp)
                    d_p = buf
                p.add_(d_p, alpha=-self.lr)
            else:
                if not st:
                    st.update(step=0, exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))
                st["step"] += 1
                b1, b2 = self.betas
                if self.wd:
                    d_p = d_p.add(p, alpha=self.wd)
                st["exp_avg"].mul_(b1).add_(d_p, alpha=1 - b1)
                st["exp_avg_sq"].mul_(b2).addcmul_(d_p, d_p, value=1 - b2)
                denom = st["exp_avg_sq"].sqrt().add_(self.eps)
                bc1, bc2 = 1 - b1 ** st["step"], 1 - b2 ** st["step"]
                p.addcdiv_(st["exp_avg"], denom, value=-self.lr * math.sqrt(bc2) / bc1)


def _params():
    torch.manual_seed(0)
    return [torch.nn.Parameter(torch.randn(37, 5)), torch.nn.Parameter(torch.randn(19)),
            torch.nn.Parameter(torch.randn(8, 8))]


def _grads(step):
    """Parameter 1 starts getting gradients at step 3, parameter 2 only on even steps."""
    g = torch.Generator().manual_seed(7 + step)
    out = [torch.randn(37, 5, generator=g), torch.randn(19, generator=g), torch.randn(8, 8, generator=g)]
    if step < 3:
        out[1] = None
    if step % 2:
        out[2] = None
    return out


KW = {"sgd": dict(lr=0.1, momentum=0.9, dampening=0.5, weight_decay=0.01),
      "adam": dict(lr=1e-2, weight_decay=0.01)}


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_late_starting_parameters_follow_reference(kind):
    import hipps

    ps, rs = _params(), _params()
    cls = hipps.SGD if kind == "sgd" else hipps.Adam
    opt = cls([(f"p{i}", p) for i, p in enumerate(ps)], mode="local", **KW[kind])
    kw = dict(KW[kind])
    ref = RefOpt(rs, kind, kw.pop("lr"), momentum=kw.get("momentum", 0), dampening=kw.get("dampening", 0),
                 wd=kw.get("weight_decay", 0))
    for s in range(7):
        gs = _grads(s)
        opt.zero_grad()
        for p, r, g in zip(ps, rs, gs):
            p.grad = None if g is None else g.clone()
            r.grad = None if g is None else g.clone()
        opt.step()
        ref.step()
        for i, (p, r) in enumerate(zip(ps, rs)):
            torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-6, atol=1e-7, msg=f"step {s} param {i}")
    # per-parameter step counts, torch-compatible state_dict entries
    assert opt.param_steps() == {0: 7, 1: 4, 2: 4}
    if kind == "adam":
        sd = opt.state_dict()
        assert [sd["state"][i]["step"] for i in range(3)] == [7, 4, 4]
    opt.close()


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(12, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))


def _data(rank, step):
    g = torch.Generator().manual_seed(100 * step + rank)
    return torch.randn(8, 12, generator=g), torch.randint(0, 3, (8,), generator=g)


def _train(rank, world, mode, kind):
    import hipps

    m = _mlp()
    cls = hipps.SGD if kind == "sgd" else hipps.Adam
    opt = cls(m.named_parameters(), mode=mode, **KW[kind])
    for s in range(4):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    return [p.detach().clone() for p in m.parameters()]


def _simulate(world, kind):
    m = _mlp()
    kw = dict(KW[kind])
    ref = RefOpt(m.parameters(), kind, kw.pop("lr"), momentum=kw.get("momentum", 0),
                 dampening=kw.get("dampening", 0), wd=kw.get("weight_decay", 0))
    for s in range(4):
        gsum = None
        for r in range(world):
            mr = _mlp()
            mr.load_state_dict(m.state_dict())
            x, y = _data(r, s)
            torch.nn.functional.cross_entropy(mr(x), y).backward()
            g = [p.grad.clone() for p in mr.parameters()]
            gsum = g if gsum is None else [a + b for a, b in zip(gsum, g)]
        for p, g in zip(m.parameters(), gsum):
            p.grad = g
        ref.step()
    return [p.detach().clone() for p in m.parameters()]


@pytest.mark.parametrize("mode", ["allgather", "ps_sync"])
def test_sync_modes_dampening_first_step_matches_reference(mode):
    """The sync engines always apply a presence mask; the first momentum step must still be
    ``buf = d_p`` (not ``(1 - dampening) * d_p``)."""
    out = run_world(_train, 2, mode, "sgd")
    want = _simulate(2, "sgd")
    for a, b, c in zip(out[0], out[1], want):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6)
