"""Drop-in import path of the reference package (``from ray_lightning import RayAccelerator``).

Everything is implemented in :mod:`ray_lightning_accelerators_amd`; this package only
re-exports the reference's public names (reference ray_lightning/__init__.py:1-4).
"""
from ray_lightning_accelerators_amd import HorovodRayAccelerator, RayAccelerator  # noqa: F401

__all__ = ["RayAccelerator", "HorovodRayAccelerator"]
