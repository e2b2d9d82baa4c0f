"""MLP for BASELINE config 1 ("2-layer MLP on MNIST, sync PS, CPU + world_size=2").

784-200-10 (159,010 params in 4 tensors, SURVEY.md §6 derived-cost table)."""
import torch.nn as nn


def mlp_mnist(hidden: int = 200, num_classes: int = 10) -> nn.Module:
    return nn.Sequential(nn.Flatten(), nn.Linear(784, hidden), nn.ReLU(), nn.Linear(hidden, num_classes))
