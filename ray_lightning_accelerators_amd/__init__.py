"""MI355X-native distributed training accelerators for Lightning-style training.

Public API (reference parity):
  * ``RayAccelerator(num_workers, num_cpus_per_worker, use_gpu, init_hook)``
  * ``HorovodRayAccelerator(num_hosts, num_slots, use_gpu)``
  * ``tune.TuneReportCallback`` / ``tune.TuneReportCheckpointCallback``
  * ``session.get_actor_rank/put_queue/init_session``
Subsystems: ``runtime`` (actor runtime), ``lightning`` (Trainer facade),
``parallel`` (flat-arena DDP, fused optimizers, fused MLP engine),
``ops`` (gfx950 HIP kernels), ``horovod`` (Horovod-compatible API),
``tune`` (sweep runner), ``models`` (MNIST classifier, BoringModel, ResNet-50).
"""
__version__ = "0.1.0"

__all__ = ["RayAccelerator", "HorovodRayAccelerator"]


def __getattr__(name):
    # lazy: runtime worker processes import this package without paying for torch
    if name == "RayAccelerator":
        from .accelerators.ray_ddp import RayAccelerator

        return RayAccelerator
    if name == "HorovodRayAccelerator":
        from .accelerators.ray_horovod import HorovodRayAccelerator

        return HorovodRayAccelerator
    raise AttributeError(name)
