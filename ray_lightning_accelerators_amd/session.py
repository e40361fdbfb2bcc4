"""Per-worker session: actor rank + handle to the driver-bound queue.

Same contract as the reference's ``ray_lightning/session.py:1-63``:
``init_session`` raises on double initialisation, ``get_session`` raises
outside a run, ``put_queue`` enqueues ``(rank, item)`` and raises if no queue
was set up.
"""
from __future__ import annotations

from typing import Any, Optional


class RayLightningSession:
    def __init__(self, rank: int, queue: Optional[Any]):
        self._rank = rank
        self._queue = queue

    def get_actor_rank(self) -> int:
        return self._rank

    def set_queue(self, queue) -> None:
        self._queue = queue

    def put_queue(self, item: Any) -> None:
        if self._queue is None:
            raise ValueError(
                "Trying to put something into the session queue, but no queue was initialised "
                "(the accelerator only creates one inside a Tune session).")
        self._queue.put((self._rank, item))


_session: Optional[RayLightningSession] = None


def init_session(*args, **kwargs) -> None:
    global _session
    if _session is not None:
        raise ValueError("Trying to initialize RayLightningSession twice.\n"
                         "FIX THIS by not calling `init_session()` manually.")
    _session = RayLightningSession(*args, **kwargs)


def shutdown_session() -> None:
    global _session
    _session = None


# a worker's last queue item: the driver's result pump (util.process_results) stops
# polling the queue once every rank sent it and waits on the results directly
WORKER_DONE = "__rla_worker_done__"


def finish_session() -> None:
    """End of a worker's run: tell the driver no queue item follows, then shut down."""
    s = _session
    if s is not None and s._queue is not None:
        try:
            s._queue.put((s._rank, WORKER_DONE))
        except Exception:  # noqa: BLE001 - the pump falls back to polling
            pass
    shutdown_session()


def get_session() -> RayLightningSession:
    if _session is None or not isinstance(_session, RayLightningSession):
        raise ValueError("Trying to access RayLightningSession from outside a training run.\n"
                         "FIX THIS by calling `get_actor_rank()` etc. only inside a worker.")
    return _session


def is_session_initialized() -> bool:
    return _session is not None


def set_session_queue(queue) -> None:
    get_session().set_queue(queue)


def get_actor_rank() -> int:
    return get_session().get_actor_rank()


def put_queue(*args, **kwargs) -> None:
    get_session().put_queue(*args, **kwargs)
