"""Loader for the in-tree native extension ``hipps._C``.

Device (HIP) tensors are ALWAYS served by the native gfx950 kernels: if the extension is
missing, the op raises instead of silently running an eager PyTorch fallback.  CPU tensors are
served by :mod:`hipps.ops.reference` (pure torch; also the numerics oracle in tests).
"""
from __future__ import annotations

import importlib
import os

_C = None
_ERR = None


def load(required: bool = False):
    """Import hipps._C (building it in-tree first if HIPPS_AUTOBUILD=1)."""
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (load torch's HIP runtime + RCCL first: same sonames)

        _C = importlib.import_module("hipps._C")
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        _ERR = e
        if os.environ.get("HIPPS_AUTOBUILD", "0") == "1":
            from hipps import _build

            _build.build()
            _C = importlib.import_module("hipps._C")
        elif required:
            raise RuntimeError(
                "hipps native extension is not built (hipps/_C*.so missing). Build it with "
                "`python -m hipps._build` (or __graft_entry__.build()). Original error: %r" % (e,)
            ) from e
    return _C


def native():
    """The extension module; raises if it cannot be loaded."""
    return load(required=True)


def available() -> bool:
    return load(required=False) is not None
