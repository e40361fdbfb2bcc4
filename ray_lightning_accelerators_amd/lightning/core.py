"""``LightningModule`` / ``LightningDataModule`` compatible base classes.

Implements the hook surface the reference's tests and examples rely on
(SURVEY.md §2.9): ``training_step`` / ``training_step_end`` /
``training_epoch_end``, ``validation_*``, ``test_*``, ``configure_optimizers``
(single optimizer or ``([opts], [scheds])``), ``*_dataloader``,
``prepare_data``, ``setup``, ``on_save_checkpoint`` / ``on_load_checkpoint``,
``on_epoch_end`` and friends, ``self.log``, ``save_hyperparameters`` and
``load_from_checkpoint``.
"""
from __future__ import annotations

import copy
import inspect
from typing import Any, Dict, List, Optional, Union

import torch
from torch import nn

from .utilities import AttributeDict, load_checkpoint


class LightningModule(nn.Module):
    CHECKPOINT_HYPER_PARAMS_KEY = "hyper_parameters"
    CHECKPOINT_HYPER_PARAMS_NAME = "hparams_name"

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.trainer = None
        self._hparams = AttributeDict()
        self._results: Dict[str, dict] = {}
        self._current_fx: Optional[str] = None
        self.exp_save_path = None

    # ----------------------------------------------------------- properties
    @property
    def hparams(self) -> AttributeDict:
        return self._hparams

    @property
    def device(self) -> torch.device:
        for p in self.parameters():
            return p.device
        for b in self.buffers():
            return b.device
        return torch.device("cpu")

    @property
    def on_gpu(self) -> bool:
        return self.device.type == "cuda"

    @property
    def global_rank(self) -> int:
        return self.trainer.global_rank if self.trainer is not None else 0

    @property
    def local_rank(self) -> int:
        return self.trainer.local_rank if self.trainer is not None else 0

    @property
    def current_epoch(self) -> int:
        return self.trainer.current_epoch if self.trainer is not None else 0

    @property
    def global_step(self) -> int:
        return self.trainer.global_step if self.trainer is not None else 0

    # ------------------------------------------------------------- hparams
    def save_hyperparameters(self, *args, frame=None) -> None:
        if frame is None:
            frame = inspect.currentframe().f_back
        init_args = inspect.getargvalues(frame)
        local = {k: init_args.locals[k] for k in init_args.args if k != "self"}
        if init_args.keywords:
            local.update(init_args.locals.get(init_args.keywords, {}))
        if args:
            if len(args) == 1 and isinstance(args[0], dict):
                local = dict(args[0])
            else:
                local = {k: local[k] for k in args if k in local}
        self._hparams.update(local)
        self._hparams_init_args = dict(local)

    # ------------------------------------------------------------- logging
    def log(self, name: str, value: Any, prog_bar: bool = False, logger: bool = True,
            on_step: Optional[bool] = None, on_epoch: Optional[bool] = None, reduce_fx=torch.mean,
            sync_dist: bool = False, sync_dist_op: str = "mean", **_kw) -> None:
        """Record a metric (rank-local unless ``sync_dist``)."""
        if self.trainer is not None:
            self.trainer._log_metric(self, name, value, prog_bar=prog_bar, logger=logger, on_step=on_step,
                                     on_epoch=on_epoch, sync_dist=sync_dist, sync_dist_op=sync_dist_op)

    def log_dict(self, dictionary: Dict[str, Any], **kwargs) -> None:
        for k, v in dictionary.items():
            self.log(k, v, **kwargs)

    def print(self, *args, **kwargs) -> None:
        if self.global_rank == 0:
            print(*args, **kwargs)

    # --------------------------------------------------------------- hooks
    def forward(self, *args, **kwargs):
        raise NotImplementedError

    def training_step(self, *args, **kwargs):
        raise NotImplementedError("training_step must be implemented")

    def training_step_end(self, outputs):
        return outputs

    def training_epoch_end(self, outputs) -> None:
        pass

    def validation_step(self, *args, **kwargs):
        return None

    def validation_step_end(self, outputs):
        return outputs

    def validation_epoch_end(self, outputs) -> None:
        pass

    def test_step(self, *args, **kwargs):
        return None

    def test_step_end(self, outputs):
        return outputs

    def test_epoch_end(self, outputs) -> None:
        pass

    def predict_step(self, batch, batch_idx, dataloader_idx=None):
        return self(batch)

    def configure_optimizers(self):
        raise NotImplementedError("configure_optimizers must be implemented")

    def train_dataloader(self):
        return None

    def val_dataloader(self):
        return None

    def test_dataloader(self):
        return None

    def prepare_data(self) -> None:
        pass

    def setup(self, stage: Optional[str] = None) -> None:
        pass

    def teardown(self, stage: Optional[str] = None) -> None:
        pass

    def on_fit_start(self): pass
    def on_fit_end(self): pass
    def on_train_start(self): pass
    def on_train_end(self): pass
    def on_epoch_start(self): pass
    def on_epoch_end(self): pass
    def on_train_epoch_start(self): pass
    def on_train_epoch_end(self, outputs=None): pass
    def on_validation_epoch_start(self): pass
    def on_validation_epoch_end(self): pass
    def on_test_epoch_start(self): pass
    def on_test_epoch_end(self): pass
    def on_train_batch_start(self, batch, batch_idx, dataloader_idx=0): pass
    def on_train_batch_end(self, outputs, batch, batch_idx, dataloader_idx=0): pass
    def on_validation_batch_start(self, batch, batch_idx, dataloader_idx=0): pass
    def on_validation_batch_end(self, outputs, batch, batch_idx, dataloader_idx=0): pass
    def on_test_batch_start(self, batch, batch_idx, dataloader_idx=0): pass
    def on_test_batch_end(self, outputs, batch, batch_idx, dataloader_idx=0): pass
    def on_before_zero_grad(self, optimizer): pass
    def on_after_backward(self): pass
    def on_save_checkpoint(self, checkpoint: dict) -> None: pass
    def on_load_checkpoint(self, checkpoint: dict) -> None: pass

    def backward(self, loss: torch.Tensor, optimizer=None, optimizer_idx: int = 0, *args, **kwargs) -> None:
        loss.backward(*args, **kwargs)

    def optimizer_step(self, epoch=None, batch_idx=None, optimizer=None, optimizer_idx=0,
                       optimizer_closure=None, **kwargs) -> None:
        optimizer.step()

    def optimizer_zero_grad(self, epoch, batch_idx, optimizer, optimizer_idx) -> None:
        optimizer.zero_grad()

    def get_progress_bar_dict(self) -> Dict[str, Any]:
        return {}

    # ------------------------------------------------------------ loading
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path: str, map_location: Any = None, strict: bool = True,
                             **kwargs):
        ckpt = load_checkpoint(checkpoint_path, map_location=map_location or "cpu")
        return cls._load_model_state(ckpt, strict=strict, **kwargs)

    @classmethod
    def _load_model_state(cls, checkpoint: dict, strict: bool = True, **cls_kwargs):
        hp = dict(checkpoint.get(cls.CHECKPOINT_HYPER_PARAMS_KEY) or {})
        hp.update(cls_kwargs)
        sig = inspect.signature(cls.__init__)
        params = list(sig.parameters.values())[1:]
        accepts_var_kw = any(p.kind == p.VAR_KEYWORD for p in params)
        names = {p.name for p in params}
        init_kw = hp if accepts_var_kw else {k: v for k, v in hp.items() if k in names}
        model = cls(**init_kw)
        model.on_load_checkpoint(checkpoint)
        model.load_state_dict(checkpoint["state_dict"], strict=strict)
        return model

    def __getstate__(self):
        d = self.__dict__.copy()
        # the trainer is re-attached on the receiving side
        d["trainer"] = None
        return d


class LightningDataModule:
    """DataModule surface used by the reference (prepare_data, setup(stage), *_dataloader)."""

    def __init__(self, train_transforms=None, val_transforms=None, test_transforms=None, dims=None):
        self.train_transforms = train_transforms
        self.val_transforms = val_transforms
        self.test_transforms = test_transforms
        self.dims = dims
        self.has_prepared_data = False
        self.has_setup_fit = False
        self.has_setup_test = False
        self.trainer = None

    def prepare_data(self, *args, **kwargs) -> None:
        pass

    def setup(self, stage: Optional[str] = None) -> None:
        pass

    def train_dataloader(self):
        raise NotImplementedError

    def val_dataloader(self):
        return None

    def test_dataloader(self):
        return None

    def transfer_batch_to_device(self, batch, device):
        from .utilities import move_to_device

        return move_to_device(batch, device)

    def size(self, dim=None):
        if dim is None or self.dims is None:
            return self.dims
        return self.dims[dim]


def _normalize_optimizers(result) -> tuple:
    """configure_optimizers() -> (optimizers, schedulers-as-dicts)."""
    if result is None:
        return [], []
    if isinstance(result, torch.optim.Optimizer):
        return [result], []
    if isinstance(result, dict):
        opt = result["optimizer"]
        sched = result.get("lr_scheduler")
        return [opt], ([_sched_dict(sched)] if sched is not None else [])
    if isinstance(result, (list, tuple)):
        if len(result) == 2 and isinstance(result[0], (list, tuple)):
            opts = list(result[0])
            scheds = [_sched_dict(s) for s in (result[1] if isinstance(result[1], (list, tuple)) else [result[1]])]
            return opts, scheds
        if all(isinstance(o, torch.optim.Optimizer) for o in result):
            return list(result), []
        if all(isinstance(o, dict) for o in result):
            opts, scheds = [], []
            for d in result:
                opts.append(d["optimizer"])
                if d.get("lr_scheduler") is not None:
                    scheds.append(_sched_dict(d["lr_scheduler"]))
            return opts, scheds
    raise ValueError(f"unsupported configure_optimizers() return value: {type(result)}")


def _sched_dict(s) -> dict:
    if isinstance(s, dict):
        d = {"interval": "epoch", "frequency": 1, "monitor": None, "reduce_on_plateau": False}
        d.update(s)
        d["scheduler"] = s["scheduler"]
        d["reduce_on_plateau"] = isinstance(d["scheduler"], torch.optim.lr_scheduler.ReduceLROnPlateau)
        return d
    return {"scheduler": s, "interval": "epoch", "frequency": 1, "monitor": "val_loss",
            "reduce_on_plateau": isinstance(s, torch.optim.lr_scheduler.ReduceLROnPlateau)}


def deepcopy_model(model: LightningModule) -> LightningModule:
    trainer = model.trainer
    model.trainer = None
    try:
        return copy.deepcopy(model)
    finally:
        model.trainer = trainer
