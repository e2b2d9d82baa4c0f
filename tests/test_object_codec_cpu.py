"""The reference's codec plug-in contract (ps.py:57, 65-66, 94, 165-166; README.md:24-31): any
object with ``encode(grad)`` / ``decode(code, cuda=)`` whose ``codes`` attribute the engine sets
before decoding.  Codes here are variable-size Python objects (a rank-r SVD of each matrix, with
r depending on the gradient), so they take the size-round + payload path in every mode."""
import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp


class SVDCodec:
    """Toy ``codings``-style codec: rank-r truncated SVD for matrices, raw tensor for vectors.
    r varies with the gradient (energy threshold), so message sizes differ per tensor, rank and
    step -- the case the reference's Iallgather size round exists for (mpi_comms.py:144-174)."""

    def __init__(self, energy=0.5, max_rank=4):
        self.energy = energy
        self.max_rank = max_rank
        self.codes = None
        self.seen_codes = 0

    def encode(self, grad):
        if grad.dim() != 2:
            return {"kind": "dense", "x": grad.detach().clone()}
        u, s, v = torch.linalg.svd(grad.detach(), full_matrices=False)
        e = torch.cumsum(s ** 2, 0) / (s ** 2).sum().clamp_min(1e-30)
        r = int(min(self.max_rank, int((e < self.energy).sum()) + 1))
        return {"kind": "svd", "u": u[:, :r].clone(), "s": s[:r].clone(), "v": v[:r].clone(), "rank": r}

    def decode(self, code, cuda=False):
        assert self.codes is not None and any(c is code for c in self.codes)  # ps.py:165 contract
        self.seen_codes = max(self.seen_codes, len(self.codes))
        if code["kind"] == "dense":
            return code["x"]
        return (code["u"] * code["s"]) @ code["v"]


def _train(rank, world, mode, steps):
    import hipps

    m = _mlp()
    code = SVDCodec()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode=mode, code=code, max_delay=0,
                    accumulate=world)
    losses, sizes = [], []
    for s in range(steps):
        x, y = _data(rank, s % 2)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        _, data = opt.step()
        losses.append(loss.item())
        sizes.append(data["msg_bytes"])
    opt.close()
    return {"params": [p.detach().clone() for p in m.parameters()], "losses": losses, "sizes": sizes,
            "seen": code.seen_codes, "prep": data.get("iallgather_prepare_time", -1)}


@pytest.mark.parametrize("mode,world", [("local", 1), ("allgather", 2), ("ps_sync", 2), ("ps_async", 2)])
def test_object_codec_trains_in_every_mode(mode, world):
    steps = 8
    out = run_world(_train, world, mode, steps)
    for r in range(world):
        L = out[r]["losses"]
        assert sum(L[-2:]) / 2 < sum(L[:2]) / 2, (mode, L)
        assert out[r]["sizes"][0] > 0
    if mode == "allgather":
        for a, b in zip(out[0]["params"], out[1]["params"]):
            assert torch.equal(a, b), "replicas diverged"
        assert out[0]["seen"] == 2  # decode saw both ranks' codes in .codes
    if mode == "ps_sync":
        for a, b in zip(out[0]["params"], out[1]["params"]):
            assert torch.equal(a, b)
    # variable sizes really vary (SVD rank follows the gradient)
    assert len(set(out[0]["sizes"])) > 1


def test_object_codec_matches_dense_sum_for_exact_codes():
    """An exact object codec (identity) through the object path equals the fp32 device path."""

    class Exact:
        codes = None

        def encode(self, g):
            return g.detach().clone()

        def decode(self, c, cuda=False):
            return c

    import hipps

    res = []
    for code in (Exact(), "fp32"):
        m = _mlp()
        opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="local", code=code)
        for s in range(3):
            x, y = _data(0, s)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
        opt.close()
        res.append([p.detach().clone() for p in m.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_object_codec_rejects_non_codec():
    from hipps.codecs import ObjectCodec

    with pytest.raises(TypeError):
        ObjectCodec(object())
