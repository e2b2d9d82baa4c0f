"""GPU: tracing (HIP events + roctx) and wire canaries on the native path."""
import pytest
import torch

import hipps

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("codec", ["bf16", "topk_int8:0.05", "threshold:0.001:0.2"])
def test_local_trace_and_canary_gpu(codec):
    run_local_trace_canary(codec, "cuda")


def run_local_trace_canary(codec, dev):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.ReLU(), torch.nn.Linear(512, 10)).to(dev)
    ref = [p.detach().clone() for p in m.parameters()]
    opt = hipps.SGD(m.named_parameters(), lr=0.05, mode="local", code=codec, trace=True, debug_canary=True,
                    bucket_mb=0.01)
    assert len(opt.engine.plan.buckets) > 1 and opt.engine.plan.guarded
    keys = {}
    for s in range(4):
        x = torch.randn(64, 256, device=dev)
        y = torch.randint(0, 10, (64,), device=dev)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        _, d = opt.step()
        keys.update(d)
    if dev == "cuda":
        torch.cuda.synchronize()
    keys.update(opt.engine.tracer.flush())
    assert keys.get("encode_ms", 0) > 0 and keys.get("update_ms", 0) > 0
    assert any(not torch.equal(a, b) for a, b in zip(ref, m.parameters()))
    opt.close()
