"""Fault injection for failure-path tests.

The reference is fail-fast only; these hooks let the tests prove it: a worker
that dies mid-training must surface on the driver as an error naming the rank,
the accelerator must tear every actor down, and no peer may hang in a
collective (the native comm engine's polls are bounded).

    RLA_FAULT_RANK=1 RLA_FAULT_STEP=3 [RLA_FAULT_KIND=raise|exit]

``raise`` raises ``InjectedFault`` inside training_step's loop on that rank at
that global step; ``exit`` kills the worker process (``os._exit(13)``), i.e.
a crash with no Python exception to report.
"""
from __future__ import annotations

import os

FAULT_ENV = ("RLA_FAULT_RANK", "RLA_FAULT_STEP", "RLA_FAULT_KIND")


class InjectedFault(RuntimeError):
    pass


def fault_env() -> dict:
    return {k: os.environ[k] for k in FAULT_ENV if k in os.environ}


def maybe_inject(rank: int, global_step: int) -> None:
    r = os.environ.get("RLA_FAULT_RANK")
    s = os.environ.get("RLA_FAULT_STEP")
    if r is None or s is None or int(r) != int(rank) or int(s) != int(global_step):
        return
    kind = os.environ.get("RLA_FAULT_KIND", "raise")
    if kind == "exit":
        os._exit(13)
    raise InjectedFault(f"injected fault on rank {rank} at step {global_step}")


def hang_watch_start(tag: str):
    """``RLA_HANG_DUMP_DIR``: every thread's Python stack is written to
    ``<dir>/stacks_<pid>_<tag>.txt`` every ``RLA_HANG_DUMP_S`` seconds (default 60)
    until :func:`hang_watch_stop` -- a worker stuck in a rendezvous, a collective or a
    device wait names the call it is in (scripts/bench_tune.py --diag-dir)."""
    d = os.environ.get("RLA_HANG_DUMP_DIR")
    if not d:
        return None
    import faulthandler

    os.makedirs(d, exist_ok=True)
    f = open(os.path.join(d, f"stacks_{os.getpid()}_{tag}.txt"), "w")
    faulthandler.dump_traceback_later(float(os.environ.get("RLA_HANG_DUMP_S", "60")), repeat=True, file=f)
    return f


def hang_watch_stop(f) -> None:
    if f is None:
        return
    import faulthandler

    faulthandler.cancel_dump_traceback_later()
    f.close()
    try:
        if os.path.getsize(f.name) == 0:
            os.remove(f.name)  # finished in time: nothing to keep
    except OSError:
        pass
