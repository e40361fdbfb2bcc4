"""Trial schedulers: FIFO (default) and asynchronous successive halving (ASHA)."""
from __future__ import annotations

import math
from collections import defaultdict
from typing import Any, Dict, Optional


class TrialScheduler:
    CONTINUE = "CONTINUE"
    STOP = "STOP"

    def __init__(self, metric: Optional[str] = None, mode: Optional[str] = None):
        self.metric = metric
        self.mode = mode

    def set_search_properties(self, metric: Optional[str], mode: Optional[str]) -> None:
        self.metric = self.metric or metric
        self.mode = self.mode or mode

    def on_trial_add(self, trial) -> None:
        pass

    def on_trial_result(self, trial, result: Dict[str, Any]) -> str:
        return self.CONTINUE

    def on_trial_complete(self, trial, result: Optional[Dict[str, Any]]) -> None:
        pass


class FIFOScheduler(TrialScheduler):
    pass


class ASHAScheduler(TrialScheduler):
    """Stop a trial at rung r if its metric is not in the top 1/reduction_factor."""

    def __init__(self, time_attr: str = "training_iteration", metric: Optional[str] = None,
                 mode: Optional[str] = None, max_t: int = 100, grace_period: int = 1, reduction_factor: float = 4):
        super().__init__(metric, mode)
        self.time_attr = time_attr
        self.max_t = max_t
        self.rf = reduction_factor
        self.rungs = []
        t = grace_period
        while t < max_t:
            self.rungs.append(t)
            t = int(math.ceil(t * reduction_factor))
        self.recorded: Dict[int, Dict[str, float]] = defaultdict(dict)

    def on_trial_result(self, trial, result: Dict[str, Any]) -> str:
        if self.metric not in result:
            return self.CONTINUE
        t = result.get(self.time_attr, 0)
        if t >= self.max_t:
            return self.STOP
        v = float(result[self.metric])
        sign = 1.0 if self.mode == "max" else -1.0
        for rung in reversed(self.rungs):
            if t < rung or trial.trial_id in self.recorded[rung]:
                continue
            rec = self.recorded[rung]
            rec[trial.trial_id] = sign * v
            vals = sorted(rec.values(), reverse=True)
            k = max(1, int(len(vals) / self.rf))
            cutoff = vals[k - 1] if len(vals) >= self.rf else None
            if cutoff is not None and sign * v < cutoff:
                return self.STOP
            break
        return self.CONTINUE


AsyncHyperBandScheduler = ASHAScheduler
