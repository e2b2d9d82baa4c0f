"""Debug subsystems on CPU: wire canaries, exchange-order race detector, and
per-phase tracing (§5.1)."""
import pytest
import torch

import hipps
from hipps.parallel.flat import GUARD_BYTE, BucketPlan, FlatStore

from dist_util import run_world


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(20, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _data(rank, s):
    g = torch.Generator().manual_seed(100 * rank + s)
    return torch.randn(8, 20, generator=g), torch.randint(0, 4, (8,), generator=g)


def test_guarded_plan_layout():
    m = _mlp()
    store = FlatStore([list(m.parameters())], device=torch.device("cpu"))
    plan = BucketPlan(store, hipps.codecs.get_codec("bf16"), 256, guard=True)
    assert plan.guarded and not plan.dense_ok and len(plan.buckets) > 1
    w = plan.new_wire()
    w.zero_()
    plan.fill_guards(w)
    assert not plan.bad_guards(w).any()
    b = plan.buckets[1]
    w[b.wire_offset + b.layout.nbytes] = 0  # a one-byte overrun of bucket 1
    assert plan.bad_guards(w).nonzero().view(-1).tolist() == [1]
    assert int(w[plan.buckets[0].wire_offset + plan.buckets[0].layout.nbytes]) == GUARD_BYTE


class _Overrun(hipps.codecs.Identity):
    """A buggy codec that writes one element past its message."""

    def encode_into(self, x, views, state):
        super().encode_into(x, views, state)
        xs = views["x"]
        raw = xs.view(torch.uint8)
        base = raw.untyped_storage().data_ptr()
        full = torch.empty(0, dtype=torch.uint8).set_(raw.untyped_storage())
        end = (raw.data_ptr() - base) + raw.numel()
        full[end] = 0


@pytest.mark.parametrize("mode", ["local"])
def test_canary_catches_codec_overrun(mode):
    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, mode=mode, code=_Overrun(torch.float32), debug_canary=True)
    x, y = _data(0, 0)
    torch.nn.functional.cross_entropy(m(x), y).backward()
    with pytest.raises(RuntimeError, match="canary"):
        opt.step()
    opt.close()


def _train(rank, world, mode, codec, steps, canary, trace):
    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode=mode, code=codec, debug_canary=canary, trace=trace,
                    debug_check_order=True, bucket_mb=0.0001)
    keys = set()
    for s in range(steps):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        _, d = opt.step()
        keys |= set(d)
    opt.close()
    return [p.detach().clone() for p in m.parameters()], sorted(keys)


@pytest.mark.parametrize("mode,codec", [("allgather", "fp32"), ("ps_sync", "topk:0.2"), ("ps_async", "bf16")])
def test_canary_mode_matches_plain(mode, codec):
    a = run_world(_train, 2, mode, codec, 3, True, True)
    b = run_world(_train, 2, mode, codec, 3, False, False)
    if mode != "ps_async":  # async interleaving is not deterministic across runs
        for pa, pb in zip(a[0][0], b[0][0]):
            torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7)
    assert "encode_ms" in a[0][1]
    assert "encode_ms" not in b[0][1]


def _mismatch(rank, world):
    m = _mlp()
    # rank 1 buckets differently -> a different exchange posting sequence
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="allgather", code="fp32", debug_check_order=True,
                    bucket_mb=0.0001 if rank == 0 else 64.0)
    x, y = _data(rank, 0)
    torch.nn.functional.cross_entropy(m(x), y).backward()
    try:
        opt.step()
    except RuntimeError as e:
        return str(e)
    finally:
        opt.close()
    return "no error"


def test_order_race_detector_flags_mismatch():
    out = run_world(_mismatch, 2)
    assert all("exchange order mismatch" in o for o in out), out


def _metrics(rank, world, path):
    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="allgather", code="int8", metrics_path=path, trace=True)
    for s in range(3):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    opt.close()
    return True


def test_metrics_jsonl_per_rank(tmp_path):
    import json

    from hipps.utils.metrics import summarize

    path = str(tmp_path / "m_{rank}.jsonl")
    run_world(_metrics, 2, path)
    for r in range(2):
        recs = [json.loads(l) for l in open(tmp_path / f"m_{r}.jsonl")]
        assert [x["step"] for x in recs] == [1, 2, 3] and all(x["rank"] == r for x in recs)
        for k in ("comm_wait", "optim_step_time", "code_wait", "grad_bytes_sent", "encode_ms", "update_ms"):
            assert k in recs[-1], k
        s = summarize(recs)
        assert s["grad_bytes_sent"] == recs[0]["grad_bytes_sent"] > 0
