"""Lightning -> Tune reporting callbacks for distributed trainers.

Same behaviour as the reference's ``ray_lightning/tune.py:24-199`` (SURVEY.md
§2.1 C9): the callbacks run inside the training WORKERS; rank 0 turns each
report (and, for checkpoints, the Lightning checkpoint dict that EVERY rank
builds) into a closure that is shipped through the session queue and
executed in the trial process, where ``tune.report`` / ``tune.checkpoint_dir``
live.  Sanity-check validations never report.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Union

from ..lightning.callbacks import Callback
from ..lightning.utilities import atomic_save
from ..session import get_actor_rank, put_queue
from . import session as tsession

_HOOKS = [
    "init_start", "init_end", "fit_start", "fit_end", "sanity_check_start", "sanity_check_end",
    "epoch_start", "epoch_end", "batch_start", "batch_end", "train_batch_start", "train_batch_end",
    "validation_batch_start", "validation_batch_end", "test_batch_start", "test_batch_end",
    "train_start", "train_end", "validation_start", "validation_end", "test_start", "test_end",
    "train_epoch_start", "train_epoch_end", "validation_epoch_start", "validation_epoch_end",
    "test_epoch_start", "test_epoch_end", "keyboard_interrupt",
]


class TuneCallback(Callback):
    """Base: ``on`` names the Lightning hooks (without ``on_``) that trigger ``_handle``."""

    def __init__(self, on: Union[str, List[str]] = "validation_end"):
        if isinstance(on, str):
            on = [on]
        for h in on:
            if h not in _HOOKS:
                raise ValueError(f"invalid trigger {h!r}; must be one of {_HOOKS}")
        self._on = list(on)

    def _handle(self, trainer, pl_module) -> None:
        raise NotImplementedError

    def __getattribute__(self, name):
        if name.startswith("on_") and name[3:] in object.__getattribute__(self, "_on"):
            handle = object.__getattribute__(self, "_handle")

            def hook(trainer, pl_module, *args, **kwargs):
                handle(trainer, pl_module)

            return hook
        return object.__getattribute__(self, name)


def _metric_value(v):
    return v.item() if hasattr(v, "item") else float(v)


class TuneReportCallback(TuneCallback):
    """Report metrics to Tune from rank 0 (list: same names; dict: {tune_name: lightning_name})."""

    def __init__(self, metrics: Union[None, str, List[str], Dict[str, str]] = None,
                 on: Union[str, List[str]] = "validation_end"):
        super().__init__(on)
        if isinstance(metrics, str):
            metrics = [metrics]
        self._metrics = metrics

    def _get_report_dict(self, trainer, pl_module) -> Optional[Dict[str, float]]:
        if trainer.running_sanity_check:
            return None
        if not self._metrics:
            return {k: _metric_value(v) for k, v in trainer.callback_metrics.items()}
        out = {}
        for key in self._metrics:
            metric = self._metrics[key] if isinstance(self._metrics, dict) else key
            out[key] = _metric_value(trainer.callback_metrics[metric])
        return out

    def _handle(self, trainer, pl_module) -> None:
        if get_actor_rank() == 0:
            report = self._get_report_dict(trainer, pl_module)
            if report is not None:
                put_queue(lambda: tsession.report(**report))


class _TuneCheckpointCallback(TuneCallback):
    """Every rank dumps the checkpoint dict; rank 0 ships it to the trial process."""

    def __init__(self, filename: str = "checkpoint", on: Union[str, List[str]] = "validation_end"):
        super().__init__(on)
        self._filename = filename

    @staticmethod
    def _create_checkpoint(checkpoint_dict: dict, global_step: int, filename: str) -> None:
        with tsession.checkpoint_dir(step=global_step) as checkpoint_dir:
            atomic_save(checkpoint_dict, os.path.join(checkpoint_dir, filename))

    def _handle(self, trainer, pl_module) -> None:
        if trainer.running_sanity_check:
            return
        checkpoint_dict = trainer.checkpoint_connector.dump_checkpoint()
        global_step = trainer.global_step
        filename = self._filename
        if get_actor_rank() == 0:
            put_queue(lambda: _TuneCheckpointCallback._create_checkpoint(checkpoint_dict, global_step, filename))


class TuneReportCheckpointCallback(TuneCallback):
    """Checkpoint, then report (Tune registers a checkpoint at the next report)."""

    def __init__(self, metrics: Union[None, str, List[str], Dict[str, str]] = None, filename: str = "checkpoint",
                 on: Union[str, List[str]] = "validation_end"):
        super().__init__(on)
        self._checkpoint = _TuneCheckpointCallback(filename, on)
        self._report = TuneReportCallback(metrics, on)

    def _handle(self, trainer, pl_module) -> None:
        self._checkpoint._handle(trainer, pl_module)
        self._report._handle(trainer, pl_module)
