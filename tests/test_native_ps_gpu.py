"""The native PS loop (csrc/runtime/psloop.cpp) against the Python PS loop (ps_async._serve).

Both implement the same AsySG-InCon protocol with per-bucket versions; with max_delay=0 and
every rank training on the same data the update sequence is deterministic, so the two loops must
produce bit-identical parameters -- for every codec the native loop decodes (dense fp32 / bf16,
int8, top-k, top-k + int8, threshold), for SGD and Adam, at one rank (M = 1: the update reads the
message straight from the mailbox slot) and three ranks on one device (M = 3: accumulator path,
peer-written slots read with system-scope acquires).
"""
import os

import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp

pytestmark = pytest.mark.gpu


def _run(rank, world, native, steps, codec, optim="sgd", bucket_mb=0.0005, slots=0, emu=0):
    import hipps

    os.environ["HIPPS_NATIVE_PS"] = "1" if native else "0"
    torch.cuda.set_device(0)
    m = _mlp().cuda()
    cls = hipps.SGD if optim == "sgd" else hipps.Adam
    kw = dict(lr=0.05, momentum=0.9, weight_decay=1e-4) if optim == "sgd" else dict(lr=1e-3, weight_decay=1e-4)
    if emu:
        kw["emulate_remote"] = emu
    opt = cls(m.named_parameters(), mode="ps_async", code=codec, bucket_mb=bucket_mb, max_delay=0,
              accumulate=world, mailbox_slots=slots, ps_granularity="bucket", **kw)
    nb = len(opt.engine.plan.buckets)
    for s in range(steps):
        if s == steps // 2:
            for g in opt.param_groups:  # a scheduler step: the native loop must see the new lr
                g["lr"] *= 0.5
        x, y = _data(0, s % 4)  # every rank: rank 0's data (order-independent sums)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
        opt.step()
    torch.cuda.synchronize()
    eng = opt.engine
    st = eng.ps_stats() if rank == 0 else {}
    opt.close()
    return {"nb": nb, "stats": st, "params": [p.detach().cpu() for p in m.parameters()],
            "state": {k: v.detach().cpu() for k, v in opt.flat_state.items()}}


@pytest.mark.parametrize("codec", ["fp32", "bf16", "int8", "topk:0.1", "topk_int8:0.1", "threshold:0.001:0.2"])
def test_native_loop_single_rank_bitwise(codec):
    a = run_world(_run, 1, True, 6, codec)[0]
    b = run_world(_run, 1, False, 6, codec)[0]
    assert a["stats"]["native_loop"] == 1 and b["stats"]["native_loop"] == 0
    assert a["stats"]["accumulated"] == b["stats"]["accumulated"] == 6
    assert a["stats"]["bucket_updates"] == b["stats"]["bucket_updates"] == 6 * a["nb"]
    for x, y in zip(a["params"], b["params"]):
        torch.testing.assert_close(x, y, rtol=0, atol=0)


@pytest.mark.parametrize("codec", ["fp32", "int8", "topk:0.1"])
def test_native_loop_three_ranks_bitwise(codec):
    a = run_world(_run, 3, True, 6, codec, timeout=300)
    b = run_world(_run, 3, False, 6, codec, timeout=300)
    assert a[0]["stats"]["native_loop"] == 1
    assert a[0]["stats"]["accumulated"] == 18 and a[0]["stats"]["version"] == 6
    for r in range(3):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def test_native_loop_adam_bitwise():
    a = run_world(_run, 1, True, 5, "fp32", "adam")[0]
    b = run_world(_run, 1, False, 5, "fp32", "adam")[0]
    assert a["stats"]["native_loop"] == 1
    for x, y in zip(a["params"], b["params"]):
        torch.testing.assert_close(x, y, rtol=0, atol=0)
    for k in b["state"]:
        torch.testing.assert_close(a["state"][k], b["state"][k], rtol=0, atol=0)


def test_native_loop_slot_reuse_bitwise():
    """2 message words per worker: every slot rewritten every second message."""
    a = run_world(_run, 3, True, 6, "fp32", "sgd", 1e-5, 2, timeout=300)
    b = run_world(_run, 3, False, 6, "fp32", "sgd", 1e-5, 2, timeout=300)
    for r in range(3):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


@pytest.mark.parametrize("codec", ["bf16", "int8"])
def test_native_loop_emulated_remote_load(codec):
    """emulate_remote=3 (the one-GPU rehearsal of remote workers' PS load: their messages batched
    with the real one, their traffic as few-workgroup HBM sweeps): the native and Python loops
    agree bit for bit, and the emulated copies leave the average gradient unchanged (a run with
    them is close to one without)."""
    a = run_world(_run, 1, True, 6, codec, "sgd", 0.0005, 0, 3)[0]
    b = run_world(_run, 1, False, 6, codec, "sgd", 0.0005, 0, 3)[0]
    c = run_world(_run, 1, True, 6, codec)[0]
    assert a["stats"]["native_loop"] == 1 and b["stats"]["native_loop"] == 0
    assert a["stats"]["bucket_updates"] == b["stats"]["bucket_updates"] == 6 * a["nb"]
    for x, y, z in zip(a["params"], b["params"], c["params"]):
        torch.testing.assert_close(x, y, rtol=0, atol=0)
        torch.testing.assert_close(x, z, rtol=1e-3, atol=5e-5)


def _ckpt(rank, world, path, native):
    import hipps
    from hipps.utils import checkpoint

    os.environ["HIPPS_NATIVE_PS"] = "1" if native else "0"
    torch.cuda.set_device(0)

    def make():
        m = _mlp().cuda()
        return m, hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="fp32",
                            bucket_mb=0.0005, max_delay=0, accumulate=world, ps_granularity="bucket")

    def train(m, opt, steps, s0):
        for s in range(s0, s0 + steps):
            x, y = _data(0, s % 4)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
            opt.step()

    m, opt = make()
    train(m, opt, 3, 0)
    checkpoint.save(opt, path, m)
    opt.close()
    m, opt = make()
    checkpoint.load(opt, path, m)
    train(m, opt, 3, 3)
    torch.cuda.synchronize()
    st = opt.engine.ps_stats() if rank == 0 else {}
    opt.close()
    return {"stats": st, "params": [p.detach().cpu() for p in m.parameters()]}


def test_native_loop_checkpoint_resume_matches_python(tmp_path):
    """save() quiesces the native loop (pause between messages) and load() restores its versions:
    the resumed native run equals the resumed Python-loop run bit for bit."""
    a = run_world(_ckpt, 2, str(tmp_path / "a"), True, timeout=300)
    b = run_world(_ckpt, 2, str(tmp_path / "b"), False, timeout=300)
    assert a[0]["stats"]["native_loop"] == 1 and a[0]["stats"]["accumulated"] == 6
    for r in range(2):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def _chunked(rank, world, chunk_mb):
    import hipps

    if chunk_mb:
        os.environ["HIPPS_IPC_CHUNK_MB"] = str(chunk_mb)
    else:
        os.environ.pop("HIPPS_IPC_CHUNK_MB", None)
    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", bucket_mb=0.0005, max_delay=0,
                    accumulate=world, ps_granularity="bucket", mailbox_slots=3)
    info = {"npc": opt.engine.npc, "nrc": opt.engine.nrc}
    for s in range(6):
        x, y = _data(0, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
        opt.step()
    torch.cuda.synchronize()
    opt.close()
    return {"info": info, "params": [p.detach().cpu() for p in m.parameters()]}


def test_chunked_publish_pull_bitwise():
    """Publish buffers in several allocations (chunks): the GPU-time bucket pull launches once per
    chunk over only the buckets that overlap it (pull.hip pull_copy_b_ptrs b0 / b1) and adopts the
    same parameters, bit for bit, as from one allocation."""
    a = run_world(_chunked, 2, 0.1, timeout=300)
    b = run_world(_chunked, 2, 0, timeout=300)
    assert a[0]["info"]["npc"] >= 3, a[0]["info"]  # (several buckets per chunk, buckets across chunks)
    for r in range(2):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def _scratch(rank, world, native):
    import hipps

    os.environ["HIPPS_NATIVE_PS"] = "1" if native else "0"
    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="bf16", bucket_mb=0.0005,
                    max_delay=0, accumulate=1, ps_granularity="bucket")
    eng = opt.engine
    info = {}
    if rank == 0:
        info = {"acc": eng.acc.numel(), "big": max(b.hi - b.lo for b in eng.plan.buckets),
                "numel": eng.store.numel, "scratch": eng._acc_scratch, "nb": len(eng.plan.buckets)}
    losses = []
    for s in range(6):
        x, y = _data(0, s % 4)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda())
        loss.backward()
        opt.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    wire_alloc = eng._wire is not None
    grad_alloc = eng.store.grad_allocated
    torch.distributed.barrier()  # every worker pushed its last message; close() drains the PS
    opt.close()
    st = opt._last_engine_stats if rank == 0 else {}
    return {"info": info, "stats": st, "losses": losses, "wire_alloc": wire_alloc, "grad_alloc": grad_alloc,
            "params": [p.detach().cpu() for p in m.parameters()]}


@pytest.mark.parametrize("native", [True, False])
def test_m1_accumulator_scratch_with_remote_workers(native):
    """accumulate=1 with per-bucket versions and three ranks: the peer-written messages go through
    ONE bucket-sized accumulator scratch (not a model-sized fp32 buffer), each applied before the
    next is accumulated; every message is counted and applied, training stays finite and close to
    the Python loop's, rank 0 (direct push) never allocates its wire image and no rank allocates
    the flat gradient buffer."""
    res = run_world(_scratch, 3, native, timeout=300)
    info, st = res[0]["info"], res[0]["stats"]
    assert info["scratch"] and info["acc"] < info["numel"] and info["acc"] >= info["big"]
    assert st["native_loop"] == (1 if native else 0)
    assert st["accumulated"] == 18 and st["bucket_updates"] == 18 * info["nb"]
    assert st.get("direct_updates", 0) == 6 * info["nb"]  # rank 0's own messages
    assert not res[0]["wire_alloc"]
    # bf16 codec, gather mode: autograd's gradients go straight into the messages on every rank
    assert not any(r["grad_alloc"] for r in res)
    for r in res:
        assert all(torch.isfinite(p).all() for p in r["params"])
        assert r["losses"][-1] < r["losses"][0]
