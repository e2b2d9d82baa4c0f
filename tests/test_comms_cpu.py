"""Reference comm-primitive parity (test_comms.py, test_mpi.py, test_iallgather.py), gloo world 2-3."""
import pytest
import torch

from dist_util import run_world


def _obj(rank):
    return {"str": "str", "rank": rank, "list": [rank] * (rank + 1), "t": torch.arange(3 + rank, dtype=torch.float32)}


def _gather_bcast(rank, W):
    from hipps.parallel import comms

    # test_comms.py:test_gather, including the irecv(*igather(...)) call form
    objs = comms.irecv(*comms.igather(_obj(rank), name=1), name=1)
    ok_g = True
    if rank == 0:
        ok_g = [o["rank"] for o in objs] == list(range(W)) and all(
            torch.equal(o["t"], torch.arange(3 + r, dtype=torch.float32)) for r, o in enumerate(objs))
    else:
        ok_g = objs is None
    # test_comms.py:test_bcast -- non-roots pass a different-length object
    obj = {"a": "a", "list": [0]} if rank == 0 else {"x": "x" * 100, "list": [1, 2, 3]}
    got = comms.irecv1(*comms.ibroadcast(obj))
    ok_b = got == {"a": "a", "list": [0]}
    # test_iallgather.py: size round + payload, sizes beyond int16
    ag = comms.Iallgather()
    big = {"rank": rank, "blob": b"x" * (40000 + rank)}
    objs = ag.allgather(big)
    ok_a = [o["rank"] for o in objs] == list(range(W)) and len(objs[-1]["blob"]) == 40000 + W - 1
    # ps.py-style pattern: prepare all sizes, then post all payloads, then recv
    from hipps.utils.serialization import format_for_send

    msgs = [format_for_send({"i": i, "r": rank})[0] for i in range(3)]
    sizes = ag.prepare(list(map(len, msgs)))
    resp = []
    for (req, count), msg in zip(sizes, msgs):
        req.Wait()
        resp.append(ag.send(msg, count))
    ok_p = all([o["i"] for o in ag.recv(*r)] == [i] * W for i, r in enumerate(resp))
    # test_mpi.py:14-21 Ialltoallv: rank r sends a different-size object to each destination d
    out = [{"src": rank, "dst": d, "pad": "y" * (100 * d + 7 * rank)} for d in range(W)]
    got = comms.irecv_alltoallv(*comms.ialltoallv(out))
    ok_t = [g["src"] for g in got] == list(range(W)) and all(
        g["dst"] == rank and len(g["pad"]) == 100 * rank + 7 * g["src"] for g in got)
    return ok_g, ok_b, ok_a, ok_p, ok_t


@pytest.mark.parametrize("W", [2, 3])
def test_reference_comm_primitives(W):
    for res in run_world(_gather_bcast, W):
        assert all(res), res


def test_serialization_roundtrip_and_compat():
    from hipps.utils import serialization as S

    obj = {"x": torch.randn(5, 3), "n": 7, "s": "abc", "l": [torch.arange(4), {"b": torch.ones(2, dtype=torch.bfloat16)}]}
    for level in (0, 1):
        back = S.loads(S.dumps(obj, level))
        assert torch.equal(back["x"], obj["x"]) and back["n"] == 7 and back["s"] == "abc"
        assert torch.equal(back["l"][0], obj["l"][0]) and back["l"][1]["b"].dtype == torch.bfloat16
    c = S.compress(b"hello" * 100, level=0)
    assert len(c) == 500 + 16 and S.decompress(c) == b"hello" * 100
    assert len(S.compress(b"hello" * 100, level=1)) < 100
    with pytest.raises(ValueError):
        S.compress(b"x", name="lz4")
    packaged, meta = S.format_for_send({"a": torch.ones(3)})
    assert meta["packaged_bytes"] == meta["msg_bytes"] + 16
    assert torch.equal(S.unformat(packaged)["a"], torch.ones(3))
    assert S.trim_msg(b"abc" + S.SENTINEL + b"zzz") == b"abc"
    assert S.bytes_of({"a": torch.ones(2, 3), "b": [torch.ones(4, dtype=torch.int8)]}) == 28
    back = S.to_torch(S.to_np({"a": torch.ones(2, dtype=torch.float64)}))
    assert back["a"].dtype == torch.float64


def _agv(rank, world):
    import torch

    from hipps.parallel import dist as hdist

    w = hdist.current()
    counts = [5, 0, 11][:world]
    inp = torch.arange(counts[rank], dtype=torch.uint8) + 10 * rank
    out = torch.full((sum(counts),), 255, dtype=torch.uint8)
    hdist.all_gather_v(out, inp, counts, w)
    g = torch.full((sum(counts),), 255, dtype=torch.uint8) if rank == 1 else None
    hdist.gather_v(g, inp, counts, w, dst=1)
    return out, g


def test_all_gather_v_and_gather_v_exact_counts():
    """Iallgatherv / Igatherv with exact per-rank counts (mpi_comms.py:88, 160-163), a zero count
    included: nothing padded, nothing lost."""
    import torch

    out = run_world(_agv, 3)
    want = torch.cat([torch.arange(5, dtype=torch.uint8), torch.arange(11, dtype=torch.uint8) + 20])
    for r in range(3):
        assert torch.equal(out[r][0], want)
    assert torch.equal(out[1][1], want)
    assert out[0][1] is None and out[2][1] is None
