"""Trial-side session: ``tune.report`` / ``tune.checkpoint_dir`` inside a trial process."""
from __future__ import annotations

import contextlib
import os
import socket
import time
from typing import Any, Dict, Optional

_trial_session: Optional["TrialSession"] = None


class TrialSession:
    def __init__(self, trial_id: str, trial_dir: str, config: Dict[str, Any], report_queue, experiment_id: str):
        self.trial_id = trial_id
        self.trial_dir = trial_dir
        self.config = config
        self.queue = report_queue
        self.experiment_id = experiment_id
        self.iteration = 0
        self.start = time.time()
        self.last = self.start
        self.pending_checkpoint: Optional[str] = None

    def report(self, **metrics) -> None:
        now = time.time()
        self.iteration += 1
        result = dict(metrics)
        result.update({
            "training_iteration": self.iteration,
            "iterations_since_restore": self.iteration,
            "time_this_iter_s": now - self.last,
            "time_total_s": now - self.start,
            "timestamp": int(now),
            "trial_id": self.trial_id,
            "experiment_id": self.experiment_id,
            "date": time.strftime("%Y-%m-%d_%H-%M-%S"),
            "hostname": socket.gethostname(),
            "node_ip": os.environ.get("RLA_NODE_IP", "127.0.0.1"),
            "pid": os.getpid(),
            "done": False,
        })
        if self.pending_checkpoint is not None:
            result["_checkpoint"] = self.pending_checkpoint
            self.pending_checkpoint = None
        self.last = now
        self.queue.put((self.trial_id, result))

    @contextlib.contextmanager
    def checkpoint_dir(self, step: Any):
        path = os.path.join(self.trial_dir, f"checkpoint_{step}")
        os.makedirs(path, exist_ok=True)
        yield path
        # registered with the NEXT report (Ray Tune semantics, reference tune.py:109-111)
        self.pending_checkpoint = path


def init_trial_session(*args, **kwargs) -> TrialSession:
    global _trial_session
    _trial_session = TrialSession(*args, **kwargs)
    return _trial_session


def shutdown_trial_session() -> None:
    global _trial_session
    _trial_session = None


def get_trial_session() -> Optional[TrialSession]:
    return _trial_session


def is_session_enabled() -> bool:
    return _trial_session is not None


def report(**metrics) -> None:
    s = _trial_session
    if s is None:
        raise ValueError("tune.report() called outside of a Tune trial")
    s.report(**metrics)


@contextlib.contextmanager
def checkpoint_dir(step: Any):
    s = _trial_session
    if s is None:
        raise ValueError("tune.checkpoint_dir() called outside of a Tune trial")
    with s.checkpoint_dir(step) as p:
        yield p


def get_trial_dir() -> Optional[str]:
    return _trial_session.trial_dir if _trial_session else None


def get_trial_id() -> Optional[str]:
    return _trial_session.trial_id if _trial_session else None
