"""Callback base + ModelCheckpoint + EarlyStopping with PL 1.1 semantics.

* ``ModelCheckpoint`` runs on every rank but only global rank 0 writes
  (SURVEY.md §5.4); with ``monitor=None`` it falls back to ``val_loss`` when
  that metric is logged (the PL 1.1 behaviour the reference's
  ``test_early_stop`` depends on: best checkpoint has ``val_epoch == 2``,
  reference tests/test_ddp.py:118-134), otherwise it keeps the latest.
* ``EarlyStopping`` counts validation checks; the stop decision is
  all-reduced across ranks so every worker stops at the same epoch
  (SURVEY.md §2.7 X5).
"""
from __future__ import annotations

import math
import os
import re
from typing import Any, Dict, Optional

import torch

from ..utils.timeline import mark

from .utilities import log, rank_zero_warn


class Callback:
    def on_init_start(self, trainer): pass
    def on_init_end(self, trainer): pass
    def setup(self, trainer, pl_module, stage: Optional[str] = None): pass
    def teardown(self, trainer, pl_module, stage: Optional[str] = None): pass
    def on_fit_start(self, trainer, pl_module): pass
    def on_fit_end(self, trainer, pl_module): pass
    def on_sanity_check_start(self, trainer, pl_module): pass
    def on_sanity_check_end(self, trainer, pl_module): pass
    def on_train_start(self, trainer, pl_module): pass
    def on_train_end(self, trainer, pl_module): pass
    def on_epoch_start(self, trainer, pl_module): pass
    def on_epoch_end(self, trainer, pl_module): pass
    def on_train_epoch_start(self, trainer, pl_module): pass
    def on_train_epoch_end(self, trainer, pl_module, outputs=None): pass
    def on_validation_epoch_start(self, trainer, pl_module): pass
    def on_validation_epoch_end(self, trainer, pl_module): pass
    def on_test_epoch_start(self, trainer, pl_module): pass
    def on_test_epoch_end(self, trainer, pl_module): pass
    def on_batch_start(self, trainer, pl_module): pass
    def on_batch_end(self, trainer, pl_module): pass
    def on_train_batch_start(self, trainer, pl_module, batch, batch_idx, dataloader_idx): pass
    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx, dataloader_idx): pass
    def on_validation_batch_start(self, trainer, pl_module, batch, batch_idx, dataloader_idx): pass
    def on_validation_batch_end(self, trainer, pl_module, outputs, batch, batch_idx, dataloader_idx): pass
    def on_test_batch_start(self, trainer, pl_module, batch, batch_idx, dataloader_idx): pass
    def on_test_batch_end(self, trainer, pl_module, outputs, batch, batch_idx, dataloader_idx): pass
    def on_validation_start(self, trainer, pl_module): pass
    def on_validation_end(self, trainer, pl_module): pass
    def on_test_start(self, trainer, pl_module): pass
    def on_test_end(self, trainer, pl_module): pass
    def on_keyboard_interrupt(self, trainer, pl_module): pass
    def on_after_backward(self, trainer, pl_module): pass
    def on_before_zero_grad(self, trainer, pl_module, optimizer): pass

    def on_save_checkpoint(self, trainer, pl_module, checkpoint=None) -> Optional[dict]:
        return None

    def on_load_checkpoint(self, callback_state: dict) -> None:
        pass

    @property
    def state_key(self) -> str:
        return type(self).__name__


class ModelCheckpoint(Callback):
    CHECKPOINT_JOIN_CHAR = "-"
    CHECKPOINT_NAME_LAST = "last"
    FILE_EXTENSION = ".ckpt"

    def __init__(self, dirpath: Optional[str] = None, filename: Optional[str] = None,
                 monitor: Optional[str] = None, verbose: bool = False, save_last: Optional[bool] = None,
                 save_top_k: Optional[int] = None, save_weights_only: bool = False, mode: str = "min",
                 period: int = 1, prefix: str = ""):
        self.dirpath = dirpath
        self.filename = filename
        self.monitor = monitor
        self._user_monitor = monitor
        self.verbose = verbose
        self.save_last = save_last
        self.save_top_k = save_top_k
        self.save_weights_only = save_weights_only
        self.mode = mode
        self.period = period
        self.prefix = prefix
        self.best_model_path = ""
        self.best_model_score: Optional[torch.Tensor] = None
        self.best_k_models: Dict[str, torch.Tensor] = {}
        self.kth_best_model_path = ""
        self.last_model_path = ""
        self.current_score = None
        self.last_global_step_saved = -1
        if mode not in ("min", "max"):
            raise ValueError(f"mode must be 'min' or 'max', got {mode}")

    # --------------------------------------------------------------- setup
    def on_pretrain_routine_start(self, trainer, pl_module) -> None:
        if self.dirpath is None:
            base = trainer.log_dir or trainer.default_root_dir
            self.dirpath = os.path.join(base, "checkpoints")

    def on_train_start(self, trainer, pl_module) -> None:
        self.on_pretrain_routine_start(trainer, pl_module)

    def on_validation_end(self, trainer, pl_module) -> None:
        if trainer.running_sanity_check:
            return
        self.save_checkpoint(trainer, pl_module)

    def on_train_end(self, trainer, pl_module) -> None:
        # no validation loop at all: keep the final weights
        if not trainer._has_val_loop and trainer.global_step != self.last_global_step_saved:
            self.save_checkpoint(trainer, pl_module)

    # -------------------------------------------------------------- saving
    def _monitor_key(self, metrics: Dict[str, Any]) -> Optional[str]:
        if self._user_monitor is not None:
            return self._user_monitor
        # PL 1.1 backward compatibility: monitor val_loss when it exists
        if "val_loss" in metrics:
            return "val_loss"
        return None

    def format_checkpoint_name(self, epoch: int, step: int, metrics: Dict[str, Any]) -> str:
        if self.filename:
            name = self.filename
            groups = re.findall(r"\{([^}:]+)(:[^}]*)?\}", name)
            vals = {"epoch": epoch, "step": step, **{k: _scalar(v) for k, v in metrics.items()}}
            for key, fmt in groups:
                v = vals.get(key, 0)
                name = name.replace("{" + key + (fmt or "") + "}", f"{key}={format(v, fmt[1:] if fmt else '')}")
        else:
            name = f"epoch={epoch}" if step is None else f"epoch={epoch}-step={step}"
        if self.prefix:
            name = self.prefix + self.CHECKPOINT_JOIN_CHAR + name
        return os.path.join(self.dirpath, name + self.FILE_EXTENSION)

    def _is_better(self, current: torch.Tensor) -> bool:
        if self.best_model_score is None:
            return True
        if self.mode == "min":
            return bool(current < self.best_model_score)
        return bool(current > self.best_model_score)

    def save_checkpoint(self, trainer, pl_module) -> None:
        epoch, step = trainer.current_epoch, trainer.global_step
        if self.period < 1 or (epoch + 1) % self.period != 0:
            return
        if step == self.last_global_step_saved and self.best_model_path:
            return
        if self.dirpath is None:
            self.on_pretrain_routine_start(trainer, pl_module)
        metrics = dict(trainer.callback_metrics)
        mark("ckpt_cb_begin")
        key = self._monitor_key(metrics)
        self.monitor = key
        top_k = self.save_top_k if self.save_top_k is not None else 1
        if key is not None and top_k != -1 and key not in metrics:
            rank_zero_warn(f"ModelCheckpoint(monitor={key!r}) not found in logged metrics")
            return
        defer = self.filename is None and getattr(trainer, "deferred_checkpoints_ok", lambda: False)()
        if defer:
            # the decision needs the monitored value, which is still being computed
            # on the device: snapshot the state there and decide / write in the
            # background once it is known -- the epoch end does not wait for the
            # device (trainer.defer_checkpoint); the default file name has no metrics
            filepath = self.format_checkpoint_name(epoch, step, {})
            value = metrics.get(key) if key is not None else None
            self.last_global_step_saved = step

            def job(resolve, vals):
                ckpt = resolve()

                def write(path):
                    if ckpt is None:
                        return  # ranks > 0: bookkeeping only (PL 1.1: rank 0 saves)
                    # the dict was dumped before this save point's decision: its
                    # ModelCheckpoint entry is refreshed with the decided state
                    if "callbacks" in ckpt:
                        ckpt["callbacks"] = dict(ckpt["callbacks"])
                        ckpt["callbacks"][self.state_key] = self.on_save_checkpoint(trainer, None)
                    trainer.write_checkpoint(ckpt, path)

                self._decide(trainer, epoch, step, key, top_k, filepath, vals[0], write)

            trainer.defer_checkpoint(job, self.save_weights_only, [value])
            return
        filepath = self.format_checkpoint_name(epoch, step, metrics)
        value = _scalar(metrics[key]) if key is not None and top_k != -1 else None
        mark("ckpt_metric_read")
        self._decide(trainer, epoch, step, key, top_k, filepath, value, lambda path: self._save(trainer, path))

    def _decide(self, trainer, epoch, step, key, top_k, filepath, value, save) -> None:
        """Top-k bookkeeping + writes for one save point (``value``: the monitored metric).

        As PL 1.1.7's ``_update_best_and_save``: the best / current fields are
        updated BEFORE the file is written, so the checkpoint's own
        ``callbacks[ModelCheckpoint]`` entry names this file as the best one and
        carries this save point's score (a resume from it restores them)."""
        if key is None or top_k == -1:
            prev = self.best_model_path
            self.best_model_path = filepath
            save(filepath)
            if prev and prev != filepath and top_k != -1:
                self._remove(trainer, prev)
        else:
            current = torch.as_tensor(float(value))
            if not torch.isfinite(current):
                current = torch.tensor(math.inf if self.mode == "min" else -math.inf)
            self.current_score = current
            if top_k > 0 and self._is_better(current):
                prev = self.best_model_path
                self.best_model_score = current
                self.best_model_path = filepath
                self.best_k_models = {filepath: current}
                self.kth_best_model_path = filepath
                save(filepath)
                if prev and prev != filepath:
                    self._remove(trainer, prev)
                if self.verbose:
                    log.warning(f"Epoch {epoch}: {key} reached {float(current):.5f}; saved {filepath}")
        if self.save_last:
            last = os.path.join(self.dirpath, self.CHECKPOINT_NAME_LAST + self.FILE_EXTENSION)
            save(last)
            self.last_model_path = last
        self.last_global_step_saved = step

    def _save(self, trainer, filepath: str) -> None:
        # background write (RLAConfig.async_checkpoint); the path bookkeeping is synchronous
        trainer.save_checkpoint(filepath, weights_only=self.save_weights_only, blocking=False)

    @staticmethod
    def _remove_file(path: str) -> None:
        if os.path.exists(path):
            try:
                os.remove(path)
            except OSError:
                pass

    def _remove(self, trainer, path: str) -> None:
        if trainer.is_global_zero:
            # ordered after the pending background writes (the file may not exist yet)
            op = getattr(trainer, "file_op", None)
            op(self._remove_file, path) if op is not None else self._remove_file(path)

    def on_save_checkpoint(self, trainer, pl_module, checkpoint=None) -> dict:
        return {"monitor": self.monitor, "best_model_score": self.best_model_score,
                "best_model_path": self.best_model_path, "current_score": self.current_score,
                "dirpath": self.dirpath}

    def on_load_checkpoint(self, callback_state: dict) -> None:
        self.best_model_score = callback_state.get("best_model_score")
        self.best_model_path = callback_state.get("best_model_path", "")


class EarlyStopping(Callback):
    mode_dict = {"min": torch.lt, "max": torch.gt}

    def __init__(self, monitor: str = "early_stop_on", min_delta: float = 0.0, patience: int = 3,
                 verbose: bool = False, mode: str = "auto", strict: bool = True):
        self.monitor = monitor
        self.min_delta = abs(min_delta)
        self.patience = patience
        self.verbose = verbose
        self.strict = strict
        if mode == "auto":
            mode = "max" if ("acc" in monitor) else "min"
        self.mode = mode
        self.wait_count = 0
        self.stopped_epoch = 0
        self.best_score = torch.tensor(math.inf if mode == "min" else -math.inf)
        if mode == "min":
            self.min_delta *= -1

    def on_validation_end(self, trainer, pl_module) -> None:
        if trainer.running_sanity_check:
            return
        self._run_early_stopping_check(trainer, pl_module)

    def _run_early_stopping_check(self, trainer, pl_module) -> None:
        metrics = trainer.callback_metrics
        if self.monitor not in metrics:
            if self.strict:
                raise RuntimeError(f"EarlyStopping monitor {self.monitor!r} not in logged metrics "
                                   f"{sorted(metrics)}")
            return
        current = torch.as_tensor(_scalar(metrics[self.monitor]))
        if self.mode_dict[self.mode](current - self.min_delta, self.best_score):
            self.best_score = current
            self.wait_count = 0
        else:
            self.wait_count += 1
        should_stop = self.wait_count >= self.patience
        # every rank must agree (reference relies on PL's all-reduced stop flag)
        should_stop = trainer.accelerator_backend.early_stopping_should_stop(should_stop) \
            if trainer.accelerator_backend is not None else should_stop
        if should_stop:
            self.stopped_epoch = trainer.current_epoch
            trainer.should_stop = True
            if self.verbose:
                log.warning(f"Epoch {trainer.current_epoch}: early stopping ({self.monitor} did not improve "
                            f"for {self.patience} checks)")

    def on_save_checkpoint(self, trainer, pl_module, checkpoint=None) -> dict:
        return {"wait_count": self.wait_count, "stopped_epoch": self.stopped_epoch,
                "best_score": self.best_score, "patience": self.patience}

    def on_load_checkpoint(self, callback_state: dict) -> None:
        self.wait_count = callback_state["wait_count"]
        self.stopped_epoch = callback_state["stopped_epoch"]
        self.best_score = callback_state["best_score"]
        self.patience = callback_state["patience"]


class LearningRateMonitor(Callback):
    """Logs the learning rate of each optimizer group at every epoch start."""

    def __init__(self, logging_interval: Optional[str] = None):
        self.logging_interval = logging_interval

    def on_train_epoch_start(self, trainer, pl_module):
        for i, opt in enumerate(trainer.optimizers):
            for j, g in enumerate(opt.param_groups):
                trainer.logged_metrics[f"lr-{type(opt).__name__}" + (f"/pg{j + 1}" if j else "")] = g["lr"]


def _scalar(v: Any) -> float:
    if isinstance(v, torch.Tensor):
        return float(v.detach().float().mean().item())
    return float(v)
