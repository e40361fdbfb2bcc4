"""Reference import path ``ray_lightning.util``."""
from ray_lightning_accelerators_amd.util import Queue, Unavailable, _handle_queue, process_results  # noqa: F401
