from .ray_ddp import RayAccelerator, RayExecutor  # noqa: F401
from .ray_horovod import HorovodRayAccelerator  # noqa: F401
