"""Async PS on the GPU: HIP-IPC mailboxes + stream-ordered doorbells.

The box has one MI355X, so multi-rank runs put every rank on cuda:0 (IPC handles opened by
other processes on the same device; gloo only for rendezvous/barriers).  The xGMI peer path is
exercised by the driver's 8-GPU bench.
"""
import pytest
import torch

from dist_util import run_world
from test_dist_cpu import _data, _mlp

pytestmark = pytest.mark.gpu


def _gpu_async(rank, world, steps, codec, accumulate, max_delay, granularity="auto"):
    import hipps

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code=codec,
                    accumulate=accumulate, max_delay=max_delay, ps_granularity=granularity)
    init = [p.detach().clone() for p in m.parameters()]
    losses = []
    for s in range(steps):
        x, y = _data(rank, s % 4)
        x, y = x.cuda(), y.cuda()
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.item())
        opt.step()
    eng = opt.engine
    has_shadow = getattr(opt.store, "shadow", None) is not None
    opt.close()
    return {"init": init, "losses": losses, "stats": eng.ps_stats(), "shadow": has_shadow,
            "params": [p.detach().clone() for p in m.parameters()]}


def test_gpu_async_single_rank_equals_local():
    import hipps

    out = run_world(_gpu_async, 1, 5, "fp32", 1, 0)
    assert not out[0]["shadow"]  # bf16_weights='auto': no conv weights, no bf16 shadow
    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="local")
    for s in range(5):
        x, y = _data(0, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
        opt.step()
    for a, b in zip(out[0]["params"], m.parameters()):
        torch.testing.assert_close(a, b.detach().cpu(), rtol=0, atol=0)


@pytest.mark.parametrize("codec", ["bf16", "int8", "topk:0.05"])
def test_gpu_async_three_ranks_same_device(codec):
    steps = 10
    out = run_world(_gpu_async, 3, steps, codec, 0, -1, timeout=300)
    st = out[0]["stats"]
    assert st["accumulated"] == 3 * steps and st["updates"] == steps
    for r in (1, 2):
        for a, b in zip(out[0]["init"], out[r]["init"]):
            assert torch.equal(a, b)
    for r in range(3):
        L = out[r]["losses"]
        assert sum(L[-3:]) / 3 < sum(L[:3]) / 3


def test_gpu_async_resnet_tiny_ssp():
    out = run_world(_gpu_resnet, 2, timeout=300)
    assert out[0]["updates"] == 4


def _gpu_resnet(rank, world):
    import torch.nn.functional as F

    import hipps
    from hipps.models import resnet_tiny

    torch.cuda.set_device(0)
    torch.manual_seed(rank)
    m = resnet_tiny().cuda().to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="bf16", max_delay=0,
                    average=True)
    x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    for _ in range(4):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
    eng = opt.engine
    opt.close()
    return eng.ps_stats()


def _gpu_sync(rank, world, mode, codec):
    import hipps

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    # fp32 parameter wire: with 'auto' (bf16 at W > 1 on GPUs) the PS rank keeps its fp32 master
    # while the others train on the bf16 broadcast, so replicas differ by design
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode=mode, code=codec, param_wire="fp32")
    for s in range(4):
        x, y = _data(rank, s)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
        opt.step()
    torch.cuda.synchronize()
    grad_mode = opt.engine.grad_mode
    opt.close()
    return [p.detach().cpu() for p in m.parameters()], grad_mode


@pytest.mark.parametrize("mode,codec", [("allgather", "bf16"), ("allgather", "topk:0.1"), ("ps_sync", "fp32")])
def test_gpu_sync_engines_replicas_identical(mode, codec):
    """Sync engines on the GPU path (multi-tensor grad gather + fused decode/update), 2 ranks on
    one device with gloo carrying the device buffers."""
    out = run_world(_gpu_sync, 2, mode, codec, timeout=300)
    assert out[0][1] == "gather"
    for a, b in zip(out[0][0], out[1][0]):
        assert torch.equal(a, b)


def _tiny_overlap(rank, world, overlap, steps, pull_shadow="1", direct_push="1"):
    import hashlib

    import torch.nn.functional as F

    import os

    import hipps
    from hipps.models import resnet_tiny

    os.environ["HIPPS_PULL_SHADOW"] = pull_shadow
    os.environ["HIPPS_DIRECT_PUSH"] = direct_push
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    m = resnet_tiny().cuda().to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="fp32", max_delay=0,
                    bf16_weights="on")
    ok = opt.overlap_pull(m.layer2) if overlap else False
    g = torch.Generator().manual_seed(1)
    losses = []
    for _ in range(steps):
        x = torch.randn(8, 3, 32, 32, generator=g).cuda().contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), generator=g).cuda()
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.item())
        opt.step()
    torch.cuda.synchronize()
    out = {"ok": ok, "losses": losses, "ver": opt.engine.adopted_version(),
           "sha": hashlib.sha1(opt.store.data.cpu().numpy().tobytes()).hexdigest(),
           "shadow": hashlib.sha1(opt.store.shadow.view(torch.int16).cpu().numpy().tobytes()).hexdigest(),
           "shadow_is_cast": torch.equal(opt.store.shadow, opt.store.data.to(torch.bfloat16)),
           "direct": opt.engine._direct_push}
    opt.close()
    return out


def test_gpu_async_pull_overlap_bitwise():
    """pull_overlap (late layers' params pulled + shadow-cast on a side stream, the late module's
    forward waits) must train bit for bit like the one-stream pull (max_delay=0: the pulled
    version is deterministic)."""
    a = run_world(_tiny_overlap, 1, True, 8)[0]
    b = run_world(_tiny_overlap, 1, False, 8)[0]
    assert a["ok"] and not b["ok"]
    assert a["losses"] == b["losses"]
    assert a["sha"] == b["sha"] and a["shadow"] == b["shadow"]
    assert a["ver"] == b["ver"] >= 7


def _gpu_bucketwise(rank, world, steps, max_delay, pull):
    import hipps

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", ps_granularity="bucket",
                    bucket_mb=0.0005, max_delay=max_delay, accumulate=world, pull=pull)
    info = dict(opt.engine.transport_info())
    nb = len(opt.engine.plan.buckets)
    losses = []
    for s in range(steps):
        x, y = _data(rank, s % 4)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda())
        loss.backward()
        losses.append(loss.item())
        opt.step()
    torch.cuda.synchronize()
    eng = opt.engine
    selb = eng._selb.cpu().tolist()
    opt.close()
    return {"stats": eng.ps_stats(), "nb": nb, "losses": losses, "info": info, "selb": selb,
            "params": [p.detach().cpu() for p in m.parameters()]}


def test_gpu_bucket_granularity_md0_equals_model_granularity():
    """Per-bucket device pulls (pull.hip k_pull_*_b) with max_delay=0 reproduce the whole-model
    update sequence bit for bit (single rank, so both equal local SGD)."""
    a = run_world(_gpu_bucketwise, 1, 5, 0, "device")
    b = run_world(_gpu_async, 1, 5, "fp32", 1, 0, "model")
    assert a[0]["nb"] >= 3
    # M = 1: every bucket update read its message straight from the mailbox slot (no accumulator)
    assert a[0]["stats"].get("direct_updates", 0) == 5 * a[0]["nb"]
    for x, y in zip(a[0]["params"], b[0]["params"]):
        torch.testing.assert_close(x, y, rtol=0, atol=0)


def test_gpu_bucket_granularity_three_ranks_device_pull():
    steps = 10
    out = run_world(_gpu_bucketwise, 3, steps, -1, "device", timeout=300)
    st = out[0]["stats"]
    nb = out[0]["nb"]
    assert out[0]["info"]["pull"] == "device"
    assert st["accumulated"] == 3 * steps and st["version"] == steps
    assert st["bucket_updates"] == nb * steps
    for r in range(3):
        adopted = out[r]["selb"][nb:]
        assert min(adopted) >= 1 and max(adopted) <= steps  # every bucket adopted a real version
        assert sum(out[r]["losses"][-3:]) < sum(out[r]["losses"][:3])


def _gpu_wgrad_side(rank, world):
    import copy

    import torch.nn.functional as F

    import hipps
    import hipps.ops.nn as hnn
    from hipps.models.resnet import Bottleneck, ResNet

    torch.cuda.set_device(0)
    torch.manual_seed(5)
    base = ResNet(Bottleneck, [1, 1], num_classes=10, width=64).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")

    def train(side, steps=3):
        hnn._WGRAD_SIDE = side
        m = copy.deepcopy(base)
        opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="fp32", max_delay=0)
        for _ in range(steps):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        opt.close()
        return [p.detach().float().cpu() for p in m.parameters()]

    train(False, 1)  # fills the per-shape kernel tuner: both runs below use the same kernels
    ref = train(False)
    ref2 = train(False)
    print("in-line run-to-run max diff", max((a - b).abs().max().item() for a, b in zip(ref, ref2)))
    side = train(True)
    return {"ref": ref, "side": side, "used": hnn.wgrad_stream(0) is not None}


def test_gpu_wgrad_side_stream_bitwise():
    """Weight gradients on the side stream (HIPPS_WGRAD_STREAM) give the training trajectory of
    in-line weight gradients: the bucket encode and step() wait for that stream (a missed wait reads
    a half-written gradient).  Not bitwise: two in-line runs already differ in the last bit of a
    few BN parameters (library kernels with atomics on the Cin=64 3x3 weight gradient)."""
    out = run_world(_gpu_wgrad_side, 1, timeout=300)[0]
    assert out["used"]
    for a, b in zip(out["ref"], out["side"]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def _slot_reuse(rank, world, steps, bucket_mb, slots, mode="ps_async", codec="fp32", granularity="model"):
    """Every rank trains on rank 0's data: identical gradients, so the PS's sum is independent of
    the order messages arrive in and runs are comparable bit for bit."""
    import hipps

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    kw = dict(mode=mode, code=codec, bucket_mb=bucket_mb)  # same buckets: same int8 blocks
    if mode == "ps_async":
        kw.update(max_delay=0, accumulate=world, mailbox_slots=slots, ps_granularity=granularity)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, **kw)
    nb = len(opt.engine.plan.buckets)
    used_slots = getattr(opt.engine, "SLOTS", None)
    for s in range(steps):
        x, y = _data(0, s % 4)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda()).backward()
        opt.step()
    torch.cuda.synchronize()
    st = opt.engine.ps_stats() if mode == "ps_async" else {}
    opt.close()
    return {"nb": nb, "slots": used_slots, "stats": st, "params": [p.detach().cpu() for p in m.parameters()]}


@pytest.mark.parametrize("codec", ["fp32", "int8"])
def test_async_slot_reuse_stress_bitwise(codec):
    """one bucket per parameter (bucket_mb=1e-5) and a 2-slot mailbox,
    so every slot is rewritten every second message.  W=1 must equal local SGD bit for bit; W=3 on one
    device (ranks 1 and 2 take the PS's acquire path for peer-written slots) must equal the same
    world with roomy default slots (2 per bucket: no reuse within a step)."""
    steps = 8
    a = run_world(_slot_reuse, 1, steps, 1e-5, 2, "ps_async", codec)[0]
    b = run_world(_slot_reuse, 1, steps, 1e-5, 2, "local", codec)[0]
    assert a["nb"] == 4 and a["slots"] == 2
    assert a["stats"]["accumulated"] == steps
    for x, y in zip(a["params"], b["params"]):
        torch.testing.assert_close(x, y, rtol=0, atol=0)
    c = run_world(_slot_reuse, 3, steps, 1e-5, 2, "ps_async", codec, timeout=300)
    d = run_world(_slot_reuse, 3, steps, 1e-5, 0, "ps_async", codec, timeout=300)
    assert c[0]["slots"] == 2 and c[0]["nb"] == 4 and d[0]["slots"] == 2 * d[0]["nb"]
    assert c[0]["stats"]["accumulated"] == 3 * steps and c[0]["stats"]["updates"] == steps
    for r in range(3):
        for x, y in zip(c[r]["params"], d[r]["params"]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)


def _budget_refused(rank, world):
    import hipps

    torch.cuda.set_device(0)
    m = _mlp().cuda()
    real = torch.cuda.mem_get_info
    torch.cuda.mem_get_info = lambda dev=None: (1 << 20, real(dev)[1])  # pretend 1 MiB is free
    try:
        hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async")
    except MemoryError as e:
        return str(e)
    finally:
        torch.cuda.mem_get_info = real
    return None


def test_gpu_async_memory_budget_refuses_before_allocating():
    """when the PS's state does not fit in the free HBM the engine raises a
    MemoryError naming every term before it allocates anything (tools/ps_budget.py computes the
    same budget offline: Llama-3-8B at W=8 does not fit co-located)."""
    msg = run_world(_budget_refused, 1)[0]
    assert msg is not None
    for term in ("mailbox", "publish", "master", "accumulator", "optimizer", "ps_dedicated"):
        assert term in msg, msg


@pytest.mark.parametrize("overlap", [False, True])
def test_gpu_async_pull_writes_shadow_bitwise(overlap):
    """The GPU-time pull writes the bf16 weight shadow in the same pass as the fp32 parameters
    (HIPPS_PULL_SHADOW, default on): bit for bit the separate cast pass (one-stream and split pull)."""
    a = run_world(_tiny_overlap, 1, overlap, 6, "1")[0]
    b = run_world(_tiny_overlap, 1, overlap, 6, "0")[0]
    assert a["shadow_is_cast"] and b["shadow_is_cast"]
    assert a["losses"] == b["losses"] and a["sha"] == b["sha"] and a["shadow"] == b["shadow"]


def test_gpu_async_direct_push_bitwise():
    """Hook-time buckets encoded straight into rank 0's mailbox ring (HIPPS_DIRECT_PUSH, default
    on) train bit for bit like the encode into the wire buffer plus the push copy."""
    a = run_world(_tiny_overlap, 1, False, 6, "1", "1")[0]
    b = run_world(_tiny_overlap, 1, False, 6, "1", "0")[0]
    assert a["direct"] and not b["direct"]
    assert a["losses"] == b["losses"] and a["sha"] == b["sha"] and a["shadow"] == b["shadow"]


def _resnet_defer(rank, world, defer, read_grads, det=True):
    import copy  # noqa: F401

    import torch.nn.functional as F

    import hipps
    from hipps.models.resnet import Bottleneck, ResNet

    torch.cuda.set_device(0)
    hipps.set_deterministic(det)
    torch.manual_seed(7)
    m = ResNet(Bottleneck, [1, 1], num_classes=10, width=64, zero_init_residual=False).cuda()
    m = m.to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="bf16", max_delay=0,
                    defer_wgrad_join=defer)
    g = torch.Generator(device="cuda").manual_seed(3)
    norms = []
    for s in range(4):
        x = torch.randn(16, 3, 64, 64, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (16,), device="cuda", generator=g)
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        if read_grads:  # a gradient read between backward and step (clipping, logging)
            opt.join_grads()
            norms.append(torch.stack([p.grad.float().norm() for p in m.parameters() if p.grad is not None]).sum().item())
        opt.step()
    torch.cuda.synchronize()
    opt.close()
    return {"params": [p.detach().cpu() for p in m.parameters()], "norms": norms}


def _resnet_defer_both(rank, world, read_grads):
    # every run in one process: the kernel tuner's picks (weight-gradient slab counts decide the
    # summation order) are shared, as they would not be across two processes; the first run only
    # warms the tuner (its first step times the candidates)
    _resnet_defer(rank, world, False, read_grads)
    return (_resnet_defer(rank, world, True, read_grads), _resnet_defer(rank, world, False, read_grads),
            _resnet_defer(rank, world, False, read_grads))


@pytest.mark.parametrize("read_grads", [False, True])
def test_gpu_deferred_wgrad_join_matches(read_grads):
    """defer_wgrad_join: no end-of-backward join of the weight-gradient side stream; the async PS's
    per-bucket encode orders every gradient read itself, so training matches the joined default
    bit for bit (under hipps.set_deterministic: MIOpen's default algorithms alone made two joined
    runs differ), and opt.join_grads() makes a read of param.grad between backward and step see
    the finished gradients.  A gradient read before the side stream finished would be off by whole
    gradients."""
    a, b, c = run_world(_resnet_defer_both, 1, read_grads)[0]
    for y, z in zip(b["params"], c["params"]):
        assert torch.equal(y, z)  # the joined default repeats itself
    for x, y in zip(a["params"], b["params"]):
        assert torch.equal(x, y), float((x - y).abs().max())
    assert a["norms"] == b["norms"]
