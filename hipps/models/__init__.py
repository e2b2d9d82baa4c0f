"""Model zoo for the BASELINE configs (random init; no checkpoints or datasets are fetched)."""
from .mlp import mlp_mnist
from .resnet import resnet18, resnet50, resnet_tiny


def build_model(name: str, **kw):
    name = name.lower()
    if name == "resnet50":
        return resnet50(**kw)
    if name == "resnet18":
        return resnet18(**kw)
    if name == "resnet_tiny":
        return resnet_tiny(**kw)
    if name in ("mlp", "mlp_mnist"):
        return mlp_mnist(**kw)
    if name.startswith("bert") or name.startswith("llama"):
        from . import transformer

        return transformer.build(name, **kw)
    raise ValueError(f"unknown model {name!r}")


__all__ = ["build_model", "mlp_mnist", "resnet18", "resnet50", "resnet_tiny"]
