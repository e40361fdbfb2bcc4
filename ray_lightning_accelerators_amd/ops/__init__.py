"""Native (HIP / gfx950) compute ops.

The kernels live in ``csrc/*.hip`` and are built in-tree into
``ray_lightning_accelerators_amd/_C*.so`` (``python -m
ray_lightning_accelerators_amd._build``).  On a machine with a GPU the native
path is the one that runs: if the extension is missing there, :func:`require`
raises instead of silently falling back to eager PyTorch.  CPU-only hosts
(the test container) use the PyTorch reference implementations in
:mod:`.reference`, which are also the numerics oracle for the GPU tests.
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

import torch

_C = None
_load_error: Optional[BaseException] = None


def _load():
    global _C, _load_error
    if _C is not None or _load_error is not None:
        return _C
    try:
        _C = importlib.import_module("ray_lightning_accelerators_amd._C")
    except BaseException as e:  # noqa: BLE001 - surfaced by require()
        _load_error = e
    return _C


def native_available() -> bool:
    """True if the gfx950 extension is importable (says nothing about a GPU)."""
    return _load() is not None


def gpu_available() -> bool:
    return torch.cuda.is_available()


def require():
    """Return the native module or raise loudly (used on every GPU code path)."""
    mod = _load()
    if mod is None:
        raise RuntimeError(
            "ray_lightning_accelerators_amd native extension (_C) is not built or failed to load: "
            f"{_load_error!r}. Build it with `python -m ray_lightning_accelerators_amd._build`."
        )
    return mod


def use_native(t: torch.Tensor) -> bool:
    """Native kernels run for GPU tensors; env RLA_DISABLE_NATIVE=1 is a debug escape hatch."""
    if not t.is_cuda:
        return False
    if os.environ.get("RLA_DISABLE_NATIVE", "0") == "1":
        return False
    require()
    return True


from .optim import fused_adam_, fused_sgd_, multi_copy, build_copy_table, scale_, sumsq  # noqa: E402
from .fused_mlp import (  # noqa: E402
    mlp_param_count,
    mlp_supported,
    mlp_train_step,
    mlp_adam_,
    mlp_refresh_shadow,
    mlp_shadow_layout,
    mlp_eval,
    mlp_unpack,
)

__all__ = [
    "native_available",
    "gpu_available",
    "require",
    "use_native",
    "fused_adam_",
    "fused_sgd_",
    "multi_copy",
    "build_copy_table",
    "scale_",
    "sumsq",
    "mlp_param_count",
    "mlp_supported",
    "mlp_train_step",
    "mlp_eval",
    "mlp_unpack",
]
