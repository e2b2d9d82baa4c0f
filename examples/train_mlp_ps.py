"""Example: BASELINE config 1 -- 2-layer MLP, MNIST-shaped synthetic data, PS training.

    python -m hipps.launch -n 2 examples/train_mlp_ps.py --mode ps_sync     # CPU, gloo
    python -m hipps.launch -n 2 examples/train_mlp_ps.py --mode ps_async --codec topk:0.05

Mirrors how the reference is meant to be used (ps.py: SGD(named_params, params, ..., code=...);
loss, data = opt.step()).
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hipps  # noqa: E402
from hipps.models import mlp_mnist  # noqa: E402
from hipps.parallel import dist as hdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="ps_sync")
    ap.add_argument("--codec", default="fp32")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args()
    world = hdist.init_from_env(backend="gloo" if a.device == "cpu" else None)
    torch.manual_seed(0)
    model = mlp_mnist().to(a.device)
    opt = hipps.SGD(model.named_parameters(), model.parameters(), lr=0.05, momentum=0.9, mode=a.mode,
                    code=a.codec, average=True)
    g = torch.Generator().manual_seed(world.rank)
    w_true = torch.randn(784, 10, generator=g.manual_seed(42))
    for step in range(a.steps):
        x = torch.randn(64, 784, generator=g)
        y = (x @ w_true).argmax(1)
        x, y = x.to(a.device), y.to(a.device)
        opt.zero_grad()
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        _, data = opt.step()
        if world.rank == 0 and step % 10 == 0:
            print(f"step {step} loss {loss.item():.4f} grad_bytes_sent {data['grad_bytes_sent']}")
    opt.close()
    if world.rank == 0:
        print(f"final loss {loss.item():.4f}")


if __name__ == "__main__":
    main()
