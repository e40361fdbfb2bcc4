"""Driver-side helpers: the worker->driver queue and the result pump.

``process_results`` replaces the reference's busy-spin loop (util.py:96-109:
``ray.wait(timeout=0)`` at 100% of a core) with a blocking drain: the driver
sleeps in the queue actor's ``get_blocking_batch`` while workers train.
Worker exceptions still surface immediately (fail-fast).
"""
from __future__ import annotations

from typing import Callable, List, Optional

from . import runtime
from .runtime.queue import Queue  # noqa: F401  (re-export, reference util.Queue)


class Unavailable:
    """No object should be an instance of this class (missing optional dependency)."""

    def __init__(self, *args, **kwargs):
        raise RuntimeError("This class should never be instantiated.")


from .session import WORKER_DONE  # every worker's last queue item (session.finish_session)


def _run_items(items) -> int:
    done = 0
    for actor_rank, item in items:
        if isinstance(item, Callable):
            item()
        elif isinstance(item, str) and item == WORKER_DONE:
            done += 1
    return done


def _handle_queue(queue) -> None:
    """Drain the queue and call every callable item (runs in the trial/driver process)."""
    _run_items(queue.drain())


def process_results(training_result_futures: List[runtime.ObjectRef], queue: Optional[Queue] = None,
                    poll_s: float = 0.2):
    not_ready = list(training_result_futures)
    done = 0
    while not_ready:
        if queue is not None and done < len(training_result_futures):
            done += _run_items(queue.get_blocking_batch(timeout=poll_s))
            ready, not_ready = runtime.wait(not_ready, num_returns=len(not_ready), timeout=0)
        else:
            ready, not_ready = runtime.wait(not_ready, num_returns=1, timeout=None)
        runtime.get(ready)  # re-raises the first worker failure right away
    if queue is not None and done < len(training_result_futures):
        _handle_queue(queue)
    return runtime.get(training_result_futures)
