"""Reference import path ``ray_lightning.session``."""
from ray_lightning_accelerators_amd.session import (  # noqa: F401
    RayLightningSession,
    get_actor_rank,
    get_session,
    init_session,
    put_queue,
    set_session_queue,
)
