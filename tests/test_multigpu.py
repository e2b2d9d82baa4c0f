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


def _tiny(rank, world, pull, steps, codec, transport="ipc"):
    import torch.nn.functional as F

    import hipps
    from hipps.models import resnet_tiny

    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    torch.manual_seed(rank)
    m = resnet_tiny().to(dev).to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", code=codec, pull=pull,
                    average=True, async_transport=transport)
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
