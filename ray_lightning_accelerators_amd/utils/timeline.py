"""Cross-process start-up timeline (SURVEY.md §5.1 tracing).

``RLA_TIMELINE=<path>``: every process of a run (driver, runtime head's
workers, Tune trials, training workers) appends ``{"t", "pid", "event"}`` JSON
lines to one file at the milestones that decide how long a short job takes:
actor creation, trainer shipping, process-group / communicator bring-up,
engine construction, first step, teardown.  ``O_APPEND`` writes of one line
are atomic, so no locking is needed.  Off (a dict lookup) when unset.
"""
from __future__ import annotations

import json
import os
import time

ENV = "RLA_TIMELINE"


def mark(event: str, **fields) -> None:
    path = os.environ.get(ENV)
    if not path:
        return
    rec = {"t": time.time(), "pid": os.getpid(), "event": event, **fields}
    line = (json.dumps(rec, default=str) + "\n").encode()
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
    try:
        os.write(fd, line)
    finally:
        os.close(fd)


def load(path: str):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]
