"""Reference import path ``ray_lightning.ray_horovod``."""
from ray_lightning_accelerators_amd.accelerators.ray_horovod import (  # noqa: F401
    CustomRayExecutor,
    HorovodRayAccelerator,
    get_executable_cls,
)

HOROVOD_AVAILABLE = True
