"""Reference import path ``ray_lightning.ray_ddp``."""
from ray_lightning_accelerators_amd.accelerators.ray_ddp import RayAccelerator, RayExecutor, setup_address  # noqa: F401
