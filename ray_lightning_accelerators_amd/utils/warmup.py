"""Background warm-up of a pooled runtime worker.

A pooled worker reports ready after ``import torch`` and the framework's modules;
the slower first-use imports (``torch.optim`` pulls in ``torch._dynamo`` on the
first optimizer, ~1 s) continue on a thread while the worker already runs its
actor (a Tune trial driver never needs them).  Anything that forks the process
calls :func:`join` first: a fork while another thread holds an import lock can
leave the child deadlocked.
"""
from __future__ import annotations

import threading
from typing import Callable, Optional

_thread: Optional[threading.Thread] = None


def start(fn: Callable[[], None]) -> None:
    global _thread

    def run():
        try:
            fn()
        except Exception:  # noqa: BLE001 - an optimisation only
            pass

    _thread = threading.Thread(target=run, name="rla-warmup", daemon=True)
    _thread.start()


def join(timeout: Optional[float] = None) -> None:
    t = _thread
    if t is not None and t.is_alive() and t is not threading.current_thread():
        t.join(timeout)
