"""CPU unit tests: flat store, bucket plan, config, codec layouts, launcher."""
import os
import subprocess
import sys

import pytest
import torch
import torch.nn as nn

import hipps
from hipps.codecs import WireLayout, get_codec
from hipps.config import PSConfig
from hipps.parallel.flat import BucketPlan, FlatStore


def test_flat_store_views_channels_last_and_grads():
    m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.Conv2d(8, 4, 1)).to(memory_format=torch.channels_last)
    before = [p.detach().clone() for p in m.parameters()]
    st = FlatStore([list(m.parameters())])
    for p, b in zip(m.parameters(), before):
        assert torch.equal(p, b)
        assert p.data_ptr() >= st.data.data_ptr()
        assert (p.data_ptr() - st.data.data_ptr()) % 64 == 0  # 16-element aligned slots
    assert m[0].weight.is_contiguous(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 8, 8).contiguous(memory_format=torch.channels_last)
    m(x).sum().backward()  # autograd hands over fresh gradient tensors (p.grad was None) ...
    assert not st.grads_attached() and all(st.presence())
    st.attach_grads()  # ... which step() copies into the flat views
    assert st.grads_attached()
    assert st.grad.abs().sum() > 0
    st.zero_grad(set_to_none=False)  # zero-filled views, still counted as gradients
    assert st.grads_attached() and all(st.presence()) and st.grad.abs().sum() == 0
    st.zero_grad()  # torch default: None -> no gradient
    assert not any(st.presence())


def test_bucket_plan_tiles_flat_buffer_and_dense_image():
    m = nn.Sequential(*[nn.Linear(64, 64) for _ in range(6)])
    st = FlatStore([list(m.parameters())])
    plan = BucketPlan(st, get_codec("bf16"), bucket_bytes=40_000)
    assert plan.buckets[0].lo == 0 and plan.buckets[-1].hi == st.numel
    for a, b in zip(plan.buckets, plan.buckets[1:]):
        assert a.hi == b.lo
    assert len(plan.buckets) > 1
    assert plan.wire_nbytes == st.numel * 2  # dense bf16 image is linear
    assert plan.ready_order[0] == len(plan.buckets) - 1  # last layers first


def test_config_env_override(monkeypatch):
    monkeypatch.setenv("HIPPS_ACCUMULATE", "7")
    monkeypatch.setenv("HIPPS_AVERAGE", "1")
    c = PSConfig.from_kwargs(mode="ps_sync")
    assert c.accumulate == 7 and c.average is True and c.mode == "ps_sync"
    with pytest.raises(ValueError):
        PSConfig.from_kwargs(mode="bogus")


def test_codec_layouts_and_bytes():
    n = 100_000
    assert get_codec("fp32").nbytes(n) == 400_000
    assert get_codec("bf16").nbytes(n) == 200_000
    assert 100_000 + 4 * 391 <= get_codec("int8").nbytes(n) <= 100_000 + 4 * 391 + 32
    k = 1000
    assert get_codec("topk:0.01").nbytes(n) == k * 8
    lay = get_codec("topk_int8:0.01").layout(n)
    assert lay.nbytes < k * 6
    for f in lay.fields:
        assert f.offset % 16 == 0
    with pytest.raises(ValueError):
        get_codec("nope")


def test_reference_object_api_roundtrip():
    c = get_codec("topk:0.5")
    g = torch.randn(4, 5)
    code = c.encode(g)
    c.codes = [code]
    d = c.decode(code)
    assert d.shape == g.shape
    nz = d != 0
    assert nz.sum() == 10 and torch.equal(d[nz], g[nz])


def test_optimizer_kwargs_routing():
    m = nn.Linear(4, 2)
    opt = hipps.Adam(m.named_parameters(), m.parameters(), lr=1e-3, betas=(0.8, 0.9), accumulate=3, mode="local")
    assert opt.cfg.accumulate == 3 and opt.param_groups[0]["betas"] == (0.8, 0.9)
    with pytest.raises(ValueError):
        hipps.SGD(m.named_parameters(), lr=0.1, optim="adam")


def test_launcher_propagates_failure(tmp_path):
    ok = tmp_path / "ok.py"
    ok.write_text("import os; print('rank', os.environ['RANK'], os.environ['WORLD_SIZE'])\n")
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(30)\n")
    r = subprocess.run([sys.executable, "-m", "hipps.launch", "-n", "2", str(ok)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and "[rank1] rank 1 2" in r.stdout
    r = subprocess.run([sys.executable, "-m", "hipps.launch", "-n", "2", str(bad)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 3


def test_global_avg_pool_channels_last_backward():
    """hipps' global average pool equals adaptive_avg_pool2d + flatten, and its input gradient
    comes back NHWC-contiguous (the fused BatchNorm backward then needs no layout copy)."""
    import torch

    from hipps.ops.nn import global_avg_pool

    x = torch.randn(3, 16, 5, 4).contiguous(memory_format=torch.channels_last).requires_grad_()
    x2 = x.detach().clone().requires_grad_()
    g = torch.randn(3, 16)
    global_avg_pool(x).backward(g)
    torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x2, 1), 1).backward(g)
    torch.testing.assert_close(x.grad, x2.grad)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)


def test_stem_routing_predicates():
    """The hipps stem path is taken only for the ResNet stem geometry on a GPU tensor (CPU tensors,
    other convolutions, odd widths and eval-mode BNs stay on the library / module path), and the
    CPU model still trains through the module fallbacks."""
    import torch.nn as nn

    from hipps.models import resnet50
    from hipps.ops import nn as hnn

    stem = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
    x = torch.randn(2, 3, 224, 224)
    assert not hnn.stem_ok(stem, x)  # CPU tensor
    assert not hnn.stem_ok(nn.Conv2d(3, 64, 3, stride=2, padding=1, bias=False), x)
    assert not hnn.stem_ok(nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=True), x)
    bn, pool = hnn.FusedBatchNorm2d(64, relu=True), hnn.MaxPool2d(3, stride=2, padding=1)
    assert not hnn.stem_block_ok(stem, bn, pool, x)
    assert hnn._pool_geom_ok(pool) and not hnn._pool_geom_ok(nn.MaxPool2d(2, 2))
    m = resnet50(num_classes=10)
    out = m(torch.randn(2, 3, 64, 64))
    out.sum().backward()
    assert m.conv1.weight.grad is not None and m.bn1.weight.grad is not None


def test_watchdog_close_joins_and_skips_completed_events():
    """a completed event is never polled (the communicator may already be gone), and
    close() joins the thread and drops pending events before the caller destroys the comm, so a
    clean shutdown cannot end in the watchdog's abort exit."""
    import threading

    from hipps.parallel.watchdog import CommWatchdog

    class Ev:
        def __init__(self, done):
            self.done = done

        def query(self):
            return self.done

    polls = []
    wd = CommWatchdog(timeout_s=100.0)
    wd.watch(Ev(True), "done-exchange", lambda: polls.append(1))
    wd._check_events()
    assert polls == [] and wd.pending() == 0

    def bad_poll():
        raise RuntimeError("ncclInvalidUsage: communicator destroyed")

    wd.watch(Ev(False), "pending-exchange", bad_poll)
    wd.close()
    assert not wd._thread.is_alive() and wd.pending() == 0
    wd._check_events()  # after close: nothing left to poll, no exit
    assert threading.current_thread().is_alive()


def test_ps_memory_budget_terms_and_engine_agree():
    """the rank-0 PS budget is computed before allocation; the shape-only
    calculator (tools/ps_budget.py) and a live engine agree term by term."""
    import hipps
    from hipps.parallel.ps_async import budget_for_shapes, ps_memory_budget
    from test_dist_cpu import _mlp

    b = ps_memory_budget(1000, W=8, slots=4, slot_bytes=4096, npub=4, pub_esz=2, opt_floats=1)
    assert b["mailbox"] == 8 * 4 * 4096 and b["publish"] == 4 * 1000 * 2
    assert b["master"] == b["accumulator"] == b["optimizer"] == 4000
    assert b["ps_total"] == sum(b[k] for k in ("mailbox", "publish", "master", "accumulator", "optimizer",
                                                  "chunk_steps"))
    assert b["total"] == b["ps_total"] + b["worker_total"]
    d = ps_memory_budget(1000, 8, 4, 4096, 4, 2, 1, colocated=False)
    assert d["worker_total"] == 0 and d["total"] == d["ps_total"] == b["ps_total"]

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, momentum=0.9, mode="ps_async", bucket_mb=0.05, code="int8")
    live = opt.engine.memory_budget()
    shp = budget_for_shapes([tuple(p.shape) for p in m.parameters()], W=1, codec="int8", bucket_mb=0.05,
                            param_wire="fp32", opt_floats=1, shadow=False, direct_push=False)  # (CPU: no direct push)
    opt.close()
    for k in ("mailbox", "publish", "master", "accumulator", "optimizer", "chunk_steps", "worker_wire",
              "worker_codec_state"):
        assert live[k] == shp[k], (k, live[k], shp[k])


def test_gradient_hold_drain_frees_only_completed_steps():
    """Engine gradient holds (gather mode): a step's gathered gradients stay referenced until the
    comm-stream event after their gathers has completed; with a host-idle task (the forward) they
    are freed a few per call, without one they are freed at the next release (bounded memory)."""
    import types
    import weakref

    from hipps.parallel.engine import Engine

    class Ev:
        def __init__(self, done):
            self.done = done

        def query(self):
            return self.done

        def synchronize(self):
            self.done = True

    e = types.SimpleNamespace(_held=__import__("collections").deque(), _drain=[], _idle_ran=False,
                              _idle_task=object(), HOLD_MAX=Engine.HOLD_MAX, DRAIN_PER_CALL=Engine.DRAIN_PER_CALL)
    release = Engine._release_held.__get__(e)
    drain = Engine._drain_some.__get__(e)
    grads = [torch.zeros(2) for _ in range(6)]
    refs = [weakref.ref(g) for g in grads]
    ev0, ev1 = Ev(False), Ev(False)
    e._held.append((ev0, grads[:3]))
    e._held.append((ev1, grads[3:]))
    del grads
    drain()  # oldest event not complete: nothing moves, nothing freed
    assert e._idle_ran and not e._drain and all(r() is not None for r in refs)
    ev0.done = True
    drain()  # moves step 0's list over and frees DRAIN_PER_CALL of it
    assert len(e._held) == 1 and sum(r() is None for r in refs[:3]) == min(3, Engine.DRAIN_PER_CALL)
    drain()
    assert all(r() is None for r in refs[:3]) and all(r() is not None for r in refs[3:])
    # no forward ran: the release frees a completed step at once
    e._idle_ran = False
    ev1.done = True
    release()
    assert not e._held and not e._drain and all(r() is None for r in refs)
    # more than HOLD_MAX pending steps: the oldest is waited for (synchronize) and released
    for _ in range(Engine.HOLD_MAX + 1):
        e._held.append((Ev(False), [torch.zeros(1)]))
    release()
    assert len(e._held) == Engine.HOLD_MAX
    release(force=True)
    assert not e._held and not e._drain


def test_native_ps_config_parses_on_cpu():
    """The native PS loop's configuration (every key psloop.cpp reads) is built and parsed for
    every codec kind and both optimizers without a GPU: NativePS's constructor only reads it (the
    loop itself runs on the GPU, tests/test_native_ps_gpu.py)."""
    import hipps
    from test_dist_cpu import _mlp

    for cls, kw in ((hipps.SGD, dict(lr=0.1, momentum=0.9)), (hipps.Adam, dict(lr=1e-3, amsgrad=True))):
        for code in ("fp32", "bf16", "int8", "topk:0.1", "topk_int8:0.1", "threshold:0.001:0.2"):
            m = _mlp()
            opt = cls(m.named_parameters(), mode="ps_async", code=code, bucket_mb=0.0005, ps_granularity="bucket", **kw)
            eng = opt.engine
            kind = eng._native_kind(eng.codec)
            assert kind is not None, code
            nat = eng.C.NativePS(eng.ctl, eng._native_config(eng.cfg, kind))
            eng._native = nat  # hyper-parameters and counters round-trip through it
            eng._push_hyper()
            st = nat.state()
            assert st["ver"] == 0 and len(st["ver_b"]) == len(eng.plan.buckets) and not nat.alive()
            eng._native = None
            del nat
            opt.close()


def test_lr_schedule_reaches_the_ps_loop_at_once(tmp_path):
    """a scheduler writing group['lr'] notifies the engine immediately (the native PS
    loop cannot read param_groups itself), and opt.load_state_dict re-arms the watch and reloads
    the hyper-parameters."""
    import hipps
    from test_dist_cpu import _mlp

    m = _mlp()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, momentum=0.9, mode="ps_async", bucket_mb=0.05)
    calls = []
    opt.engine._push_hyper = lambda: calls.append(opt.param_groups[0]["lr"])
    reloads = []
    opt.engine.reload_hyper = lambda: reloads.append(1)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    opt.step()
    sched.step()
    assert calls and calls[-1] == pytest.approx(0.05)
    n = len(calls)
    opt.param_groups[0]["lr"] = 0.05  # same value: no push
    assert len(calls) == n
    sd = opt.state_dict()
    assert type(sd["param_groups"][0]) is dict
    opt.load_state_dict(sd)
    assert reloads == [1]
    opt.param_groups[0]["momentum"] = 0.5
    assert len(calls) == n + 1
    opt.close()


def test_tuner_picks_round_trip(tmp_path):
    """Recorded kernel picks load back (set_deterministic across processes)."""
    from hipps.ops.nn import _Tuner

    t = _Tuner()
    t.cache[("lfwd", 1024, 768, 768, True, False)] = "g2_256x256"
    t.cache[("bnpro", 256, 64, 56, 56, 256)] = False
    f = str(tmp_path / "picks.json")
    t.save(f)
    u = _Tuner()
    assert u.load(f) == 2 and u.cache == t.cache
    assert u.pick(("lfwd", 1024, 768, 768, True, False), {"x": None, "y": None}) == "g2_256x256"
