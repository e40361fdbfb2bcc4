"""Built-in actor runtime: the Ray-core subset the reference uses.

Processes: a driver, one head (node daemon: resources, actor table, spawning)
and one process per actor.  GPU actors are pinned with HIP_VISIBLE_DEVICES /
CUDA_VISIBLE_DEVICES.  Control plane only -- no training-step traffic.
"""
from .client import (  # noqa: F401
    ActorClass,
    ActorHandle,
    ObjectRef,
    RemoteFunction,
    actors,
    available_resources,
    cluster_resources,
    get,
    get_actor_id,
    get_gpu_ids,
    get_node_address,
    get_node_ip_address,
    init,
    is_initialized,
    kill,
    nodes,
    prewarm_gpu_workers,
    put,
    remote,
    shutdown,
    wait,
)
from .protocol import ActorDiedError, GetTimeoutError, RemoteError  # noqa: F401
from .queue import Empty, Full, Queue  # noqa: F401

ALIVE = "ALIVE"
DEAD = "DEAD"


class _ActorTableData:
    """``ray.gcs_utils.ActorTableData.DEAD`` compatibility (reference tests/test_ddp.py:41-42)."""

    ALIVE = ALIVE
    DEAD = DEAD
    PENDING_CREATION = "PENDING_CREATION"


class gcs_utils:  # noqa: N801 - mirrors ray.gcs_utils
    ActorTableData = _ActorTableData


class services:  # noqa: N801 - mirrors ray.services.get_node_ip_address
    get_node_ip_address = staticmethod(get_node_ip_address)
