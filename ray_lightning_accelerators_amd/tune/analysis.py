"""Trial records and ``ExperimentAnalysis`` (``best_config``, ``results_df``,
``best_checkpoint`` -- the attributes the reference's tests/examples use)."""
from __future__ import annotations

import csv
import json
import math
import os
from typing import Any, Dict, List, Optional



class Trial:
    def __init__(self, trial_id: str, config: Dict[str, Any], index: int):
        self.trial_id = trial_id
        self.config = config
        self.index = index
        self.status = "PENDING"
        self.results: List[Dict[str, Any]] = []
        self.last_result: Optional[Dict[str, Any]] = None
        self.checkpoints: List[tuple] = []  # (path, result)
        self.logdir: Optional[str] = None
        self.error: Optional[str] = None
        self.actor = None
        self.future = None
        self.stop_requested = False
        self.start_time = self.end_time = None

    def add_result(self, result: Dict[str, Any], checkpoint: Optional[str]) -> None:
        self.results.append(result)
        self.last_result = result
        if checkpoint:
            self.checkpoints.append((checkpoint, result))
        if self.logdir:
            with open(os.path.join(self.logdir, "result.json"), "a") as f:
                f.write(json.dumps(result, default=repr) + "\n")

    @property
    def checkpoint(self) -> Optional[str]:
        return self.checkpoints[-1][0] if self.checkpoints else None

    def write_logs(self) -> None:
        if not self.logdir or not self.results:
            return
        flat = [_flatten(r) for r in self.results]
        keys = []
        for r in flat:
            for k in r:
                if k not in keys:
                    keys.append(k)
        with open(os.path.join(self.logdir, "progress.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            w.writerows(flat)

    def __repr__(self) -> str:
        return f"Trial({self.trial_id}, {self.status})"


def _flatten(d: Dict[str, Any], prefix: str = "") -> Dict[str, Any]:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "/"))
        else:
            out[key] = v
    return out


def _better(a: float, b: float, mode: str) -> bool:
    if b is None or (isinstance(b, float) and math.isnan(b)):
        return True
    return a < b if mode == "min" else a > b


class ExperimentAnalysis:
    def __init__(self, experiment_dir: str, trials: List[Trial], default_metric: Optional[str] = None,
                 default_mode: Optional[str] = None):
        self.experiment_dir = experiment_dir
        self._experiment_dir = experiment_dir
        self.trials = trials
        self.default_metric = default_metric
        self.default_mode = default_mode

    # -------------------------------------------------------------- helpers
    def _mm(self, metric, mode):
        metric = metric or self.default_metric
        mode = mode or self.default_mode
        if metric is None or mode is None:
            raise ValueError("metric and mode must be given (here or to tune.run)")
        return metric, mode

    def get_best_trial(self, metric: Optional[str] = None, mode: Optional[str] = None, scope: str = "last"):
        metric, mode = self._mm(metric, mode)
        best, best_v = None, None
        for t in self.trials:
            if not t.results:
                continue
            vals = [r[metric] for r in t.results if metric in r]
            if not vals:
                continue
            if scope == "last":
                v = vals[-1]
            elif scope == "all":
                v = min(vals) if mode == "min" else max(vals)
            else:
                v = vals[-1]
            if best is None or _better(v, best_v, mode):
                best, best_v = t, v
        return best

    def get_best_config(self, metric: Optional[str] = None, mode: Optional[str] = None, scope: str = "last"):
        t = self.get_best_trial(metric, mode, scope)
        return t.config if t else None

    def get_best_logdir(self, metric: Optional[str] = None, mode: Optional[str] = None, scope: str = "last"):
        t = self.get_best_trial(metric, mode, scope)
        return t.logdir if t else None

    def get_best_checkpoint(self, trial: Trial, metric: Optional[str] = None, mode: Optional[str] = None):
        metric, mode = self._mm(metric, mode)
        best, best_v = None, None
        for path, r in trial.checkpoints:
            v = r.get(metric)
            if v is None:
                continue
            if best is None or _better(v, best_v, mode):
                best, best_v = path, v
        return best

    def get_trial_checkpoints_paths(self, trial: Trial, metric: Optional[str] = None):
        metric = metric or self.default_metric or "training_iteration"
        return [(p, r.get(metric)) for p, r in trial.checkpoints]

    # ------------------------------------------------------------ properties
    @property
    def best_trial(self) -> Optional[Trial]:
        return self.get_best_trial()

    @property
    def best_config(self) -> Optional[Dict[str, Any]]:
        return self.get_best_config()

    @property
    def best_logdir(self) -> Optional[str]:
        return self.get_best_logdir()

    @property
    def best_checkpoint(self) -> Optional[str]:
        t = self.best_trial
        return self.get_best_checkpoint(t) if t else None

    @property
    def best_result(self) -> Optional[Dict[str, Any]]:
        t = self.best_trial
        return t.last_result if t else None

    @property
    def results(self) -> Dict[str, Dict[str, Any]]:
        return {t.trial_id: t.last_result for t in self.trials}

    @property
    def results_df(self) -> "pd.DataFrame":
        rows = []
        for t in self.trials:
            if t.last_result is None:
                continue
            rows.append(_flatten(t.last_result, "") | {})
        import pandas as pd  # lazy: 0.6 s of import that trial / training workers never need

        df = pd.DataFrame([_flatten_config(r) for r in rows])
        if "trial_id" in df.columns:
            df = df.set_index("trial_id", drop=False)
        return df

    def dataframe(self, metric: Optional[str] = None, mode: Optional[str] = None) -> "pd.DataFrame":
        rows = []
        for t in self.trials:
            if not t.results:
                continue
            if metric and mode:
                vals = [r for r in t.results if metric in r]
                r = (min if mode == "min" else max)(vals, key=lambda x: x[metric]) if vals else t.last_result
            else:
                r = t.last_result
            row = _flatten_config(_flatten(r))
            row["logdir"] = t.logdir
            rows.append(row)
        import pandas as pd

        return pd.DataFrame(rows)

    def trial_dataframes(self) -> Dict[str, "pd.DataFrame"]:
        import pandas as pd

        return {t.logdir: pd.DataFrame([_flatten_config(_flatten(r)) for r in t.results]) for t in self.trials}

    def stats(self) -> Dict[str, Any]:
        return {"num_trials": len(self.trials),
                "status": {s: sum(t.status == s for t in self.trials) for s in {t.status for t in self.trials}}}


def _flatten_config(row: Dict[str, Any]) -> Dict[str, Any]:
    """Ray Tune's results_df uses ``config.<key>`` (dot-separated) columns."""
    out = {}
    for k, v in row.items():
        out[k.replace("/", ".")] = v
    return out
