"""Async PS across GPUs: one rank per device, HIP-IPC mailboxes over xGMI.

Skipped unless the box has >= 2 HIP devices (the development pool has one; the driver's 8-GPU
node runs it).  Covers the cross-device paths the same-device tests cannot:
  * peer-mapped mailbox: every rank's tensor() view of the PS's HBM carries the rank's own
    device label and the self-test's push + pull round trip passes over xGMI;
  * push / ack / GPU-time pull across devices, with device doorbells;
  * host-chosen prefetch pull across devices (side stream, reader-protected);
  * ResNet-tiny, 10 steps: the PS accounts every pushed step exactly once
    (accumulated == W * steps) and workers' adopted versions advance.
"""
import pytest
import torch

from dist_util import run_world

NDEV = torch.cuda.device_count() if torch.cuda.is_available() else 0
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(NDEV < 2, reason="needs >= 2 HIP devices")]


def _tiny(rank, world, pull, steps, codec, transport="ipc", bucket_mb=64.0, slots=0, comm="torch"):
    import torch.nn.functional as F

    import hipps
    from hipps.models import resnet_tiny

    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    torch.manual_seed(rank)
    m = resnet_tiny().to(dev).to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code=codec, pull=pull,
                    average=True, async_transport=transport, bucket_mb=bucket_mb, mailbox_slots=slots,
                    transport=comm)
    eng = opt.engine
    info = dict(eng.transport_info())
    info["mem_device"] = eng.mem.device.index if eng.mem is not None else rank
    x = torch.randn(8, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    vers = []
    for _ in range(steps):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        _, data = opt.step()
        vers.append(data["version"])
    torch.cuda.synchronize()
    opt.close()
    info.update(stats=eng.ps_stats(), versions=vers, finite=bool(torch.isfinite(loss).item()))
    return info


@pytest.mark.parametrize("pull,codec,transport", [("device", "bf16", "ipc"), ("prefetch", "bf16", "ipc"),
                                                  ("device", "topk_int8:0.05", "ipc"), ("device", "bf16", "p2p")])
def test_async_ps_across_devices(pull, codec, transport):
    W = min(NDEV, 4)
    steps = 10
    out = run_world(_tiny, W, pull, steps, codec, transport, timeout=600, backend="nccl")
    st = out[0]["stats"]
    assert st["accumulated"] == W * steps, st
    assert st["updates"] == steps  # accumulate = W
    for r, o in enumerate(out):
        assert o["mem_device"] == r  # the peer mapping is addressed from the rank's own device
        assert o["doorbells"] == "device"
        assert o["finite"]
        assert o["versions"][-1] > 0
        if pull == "device" and transport == "ipc":
            assert o["pull"] == "device"
        assert o["transport"] == transport


def test_async_p2p_on_native_rccl_split_channels():
    """the p2p transport's gradient and parameter channels as two communicators
    split from hipps' own RCCL communicator (ncclCommSplit) instead of torch process groups."""
    W = min(NDEV, 4)
    steps = 10
    out = run_world(_tiny, W, "device", steps, "bf16", "p2p", 64.0, 0, "rccl", timeout=600, backend="nccl")
    st = out[0]["stats"]
    assert st["accumulated"] == W * steps and st["updates"] == steps
    for o in out:
        assert o["transport"] == "p2p" and o["p2p_channels"] == "rccl-split" and o["finite"]


@pytest.mark.parametrize("codec", ["fp32", "int8", "topk:0.05"])
def test_async_ps_across_devices_small_buckets_slot_reuse(codec):
    """tiny buckets and a 2-slot mailbox, so a peer rewrites each slot every
    second message over xGMI while the PS's L2 may still hold the previous message's lines; the PS
    kernels' system-scope acquire (csrc/common.h) must make every message count exactly once."""
    W = min(NDEV, 4)
    steps = 10
    out = run_world(_tiny, W, "device", steps, codec, "ipc", 0.02, 2, timeout=600, backend="nccl")
    st = out[0]["stats"]
    assert st["accumulated"] == W * steps, st
    assert st["updates"] == steps
    for o in out:
        assert o["finite"] and o["versions"][-1] > 0


def _sync(rank, world, mode, transport, codec):
    """allgather / ps_sync across devices: replicas must be bitwise identical."""
    import torch.nn.functional as F

    import hipps
    from hipps.models import resnet_tiny

    dev = torch.device("cuda", rank)
    torch.manual_seed(0)
    m = resnet_tiny().to(dev).to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, dampening=0.1, mode=mode, code=codec,
                    transport=transport, param_wire="fp32", average=True)
    g = torch.Generator(device="cpu").manual_seed(rank)
    x = torch.randn(8, 3, 32, 32, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g).to(dev)
    for _ in range(4):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    opt.close()
    return [p.detach().float().cpu() for p in m.parameters()]


@pytest.mark.parametrize("mode", ["allgather", "ps_sync"])
@pytest.mark.parametrize("transport", ["torch", "rccl"])
@pytest.mark.parametrize("codec", ["bf16", "topk_int8:0.05"])
def test_sync_modes_across_devices_bitwise_replicas(mode, transport, codec):
    W = min(NDEV, 4)
    out = run_world(_sync, W, mode, transport, codec, timeout=600, backend="nccl")
    for r in range(1, W):
        for a, b in zip(out[0], out[r]):
            assert torch.equal(a, b), f"rank {r} diverged ({mode}, {transport}, {codec})"


def _rccl_v(rank, world):
    from hipps.parallel import dist as hdist
    from hipps.parallel.rccl import RcclGroup

    dev = torch.device("cuda", rank)
    g = RcclGroup(hdist.current(), dev)
    counts = [(7 * r + 3) % 11 for r in range(world)]  # includes a zero count at rank 1
    displs = [sum(counts[:r]) for r in range(world)]
    inp = (torch.arange(counts[rank], device=dev, dtype=torch.int32) + 100 * rank)
    out = torch.full((sum(counts),), -1, dtype=torch.int32, device=dev)
    g.all_gather_v(out, inp, counts, displs)
    gat = torch.full((sum(counts),), -1, dtype=torch.int32, device=dev) if rank == 0 else None
    g.gather_v(gat, inp, counts, displs, 0)
    torch.cuda.synchronize()
    g.poll()
    g.close()
    return out.cpu(), None if gat is None else gat.cpu(), counts


def test_rccl_all_gather_v_and_gather_v_across_devices():
    W = min(NDEV, 4)
    out = run_world(_rccl_v, W, timeout=300, backend="nccl")
    counts = out[0][2]
    want = torch.cat([torch.arange(c, dtype=torch.int32) + 100 * r for r, c in enumerate(counts)])
    for r in range(W):
        assert torch.equal(out[r][0], want)
    assert torch.equal(out[0][1], want)


def _p2p_collectives(rank, world):
    """p2p async transport: the PS thread serves pair send/recv while rank 0's main thread runs
    all_reduce + barrier on the default RCCL group every step."""
    import torch.distributed as dist
    import torch.nn.functional as F

    import hipps
    from hipps.models import resnet_tiny

    dev = torch.device("cuda", rank)
    m = resnet_tiny().to(dev).to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="bf16",
                    async_transport="p2p", average=True)
    x = torch.randn(8, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    for _ in range(12):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            F.cross_entropy(m(x), y).backward()
        opt.step()
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        assert t.item() == world
        dist.barrier(device_ids=[rank])
    torch.cuda.synchronize()
    eng = opt.engine
    opt.close()
    return eng.ps_stats()


def test_p2p_transport_with_main_thread_collectives_across_devices():
    W = min(NDEV, 4)
    out = run_world(_p2p_collectives, W, timeout=600, backend="nccl")
    assert out[0]["accumulated"] == 12 * W


def _dedicated(rank, world):
    import torch.nn.functional as F

    import hipps
    from hipps.models import resnet_tiny

    dev = torch.device("cuda", rank)
    m = resnet_tiny().to(dev).to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code="bf16", ps_dedicated=True,
                    average=True)
    if opt.ps_only:
        return opt.serve(timeout_s=300)
    x = torch.randn(8, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    for _ in range(10):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            F.cross_entropy(m(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    opt.close()
    return None


def test_dedicated_ps_across_devices():
    W = min(NDEV, 4)
    out = run_world(_dedicated, W, timeout=600, backend="nccl")
    assert out[0]["accumulated"] == 10 * (W - 1) and out[0]["updates"] == 10
