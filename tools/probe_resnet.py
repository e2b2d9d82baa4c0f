"""GPU probe: ResNet-50 train-step throughput under different precision/layout choices.

Used once to pick the worker compute configuration for bench.py (results -> profiles/).
"""
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from hipps.models.resnet import resnet50  # noqa: E402


def run(variant, batch, steps=12, warmup=4):
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = resnet50().to(dev)
    cl = "cl" in variant
    if cl:
        m = m.to(memory_format=torch.channels_last)
    pure_bf16 = "bf16w" in variant
    if pure_bf16:
        m = m.to(torch.bfloat16)
    x = torch.randn(batch, 3, 224, 224, device=dev)
    if pure_bf16:
        x = x.to(torch.bfloat16)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=dev)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)

    def step():
        opt.zero_grad(set_to_none=True)
        if pure_bf16:
            loss = F.cross_entropy(m(x).float(), y)
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    return {"variant": variant, "batch": batch, "ms": dt * 1e3, "img_s": batch / dt}


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0), flush=True)
    out = []
    for variant, batch in [("amp_nchw", 256), ("amp_cl", 256), ("bf16w_cl", 256), ("amp_cl", 128), ("amp_cl", 512)]:
        try:
            r = run(variant, batch)
        except Exception as e:  # keep probing other variants
            r = {"variant": variant, "batch": batch, "error": repr(e)[:300]}
        print(json.dumps(r), flush=True)
        out.append(r)
    with open("gpurun_out/probe_resnet.json", "w") as f:
        json.dump(out, f, indent=1)
