"""Shared test fixtures (same contract as the reference's ray_lightning/tests/utils.py)."""
from typing import List, Optional

import torch

import ray_lightning_accelerators_amd.lightning as pl
from ray_lightning_accelerators_amd.lightning import Callback, LightningDataModule, LightningModule, Trainer
from ray_lightning_accelerators_amd.models.boring import BoringModel  # noqa: F401
from ray_lightning_accelerators_amd.models.data import RandomDataset  # noqa: F401


def get_trainer(dir, accelerator, use_gpu: bool = False, max_epochs: int = 1, limit_train_batches=10,
                limit_val_batches=10, progress_bar_refresh_rate: int = 0,
                callbacks: Optional[List[Callback]] = None, **kwargs) -> Trainer:
    callbacks = [] if not callbacks else callbacks
    return pl.Trainer(default_root_dir=str(dir), gpus=1 if use_gpu else 0, max_epochs=max_epochs,
                      limit_train_batches=limit_train_batches, limit_val_batches=limit_val_batches,
                      progress_bar_refresh_rate=progress_bar_refresh_rate, checkpoint_callback=True,
                      callbacks=callbacks, accelerator=accelerator, **kwargs)


def train_test(trainer: Trainer, model: LightningModule) -> None:
    """Training must change the DRIVER's model weights and fit() must return 1."""
    initial = torch.tensor([torch.sum(torch.abs(x)) for x in model.parameters()])
    result = trainer.fit(model)
    post = torch.tensor([torch.sum(torch.abs(x)) for x in model.parameters()])
    assert result == 1, "trainer failed"
    assert torch.norm(initial - post) > 0.1


def load_test(trainer: Trainer, model: LightningModule) -> None:
    trainer.fit(model)
    trained = BoringModel.load_from_checkpoint(trainer.checkpoint_callback.best_model_path)
    assert trained is not None, "loading model failed"


def predict_test(trainer: Trainer, model: LightningModule, dm: LightningDataModule) -> None:
    trainer.fit(model, datamodule=dm)
    dm.setup(stage="test")
    acc = pl.metrics.Accuracy()
    for x, y in dm.test_dataloader():
        with torch.no_grad():
            y_hat = model(x)
        acc.update(y_hat.cpu(), y)
    average_acc = acc.compute()
    assert average_acc >= 0.5, f"expected > 0.5 test accuracy, got {average_acc}"


def update_worst(worst: dict, errs: dict) -> None:
    """Fold one step's per-tensor errors into running maxima WITHOUT losing a NaN:
    Python's max(0.0, nan) is 0.0, so a non-finite error is recorded as +inf (which
    no bound accepts) instead of being silently dropped."""
    import math

    for k, e in errs.items():
        e = float(e)
        worst[k] = math.inf if not math.isfinite(e) else max(worst[k], e)
