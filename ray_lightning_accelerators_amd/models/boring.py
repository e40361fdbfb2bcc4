"""``BoringModel``: the smallest LightningModule the test-suite trains.

Behavioural contract (the reference's test fixture, ray_lightning/tests/utils.py:24-91,
is what the ported tests assume): one ``Linear(32, 2)``; the training / test loss is
the MSE of the prediction against ones; validation logs a constant ``val_loss`` of
1.0 and counts finished validation epochs in ``val_epoch``, which survives a
checkpoint round trip; SGD at lr 0.1 with a per-epoch ``StepLR``; every loader is 64
random 32-vectors, batch size 1.  Step outputs keep the fixture's keys (``loss`` /
``x`` / ``y``) because Trainer callbacks and tests read them.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

from ..lightning import LightningModule
from .data import RandomDataset

_IN, _OUT, _LEN = 32, 2, 64


def _to_ones(pred: torch.Tensor) -> torch.Tensor:
    return F.mse_loss(pred, torch.ones_like(pred))


class BoringModel(LightningModule):
    def __init__(self):
        super().__init__()
        self.layer = torch.nn.Linear(_IN, _OUT)
        self.val_epoch = 0

    def forward(self, x):
        return self.layer(x)

    # kept for API parity with the fixture (some user code calls them directly)
    def loss(self, batch, prediction):
        return _to_ones(prediction)

    def step(self, x):
        return _to_ones(self(x))

    # --------------------------------------------------------------- loops
    def training_step(self, batch, batch_idx):
        return {"loss": self.step(batch)}

    def validation_step(self, batch, batch_idx):
        self(batch)  # the forward runs; the logged value does not depend on it
        val = torch.tensor(1.0)
        self.log("val_loss", val)
        return {"x": val}

    def validation_epoch_end(self, outputs) -> None:
        self.val_epoch += 1

    def test_step(self, batch, batch_idx):
        return {"y": self.step(batch)}

    # --------------------------------------------------------------- setup
    def configure_optimizers(self):
        opt = torch.optim.SGD(self.layer.parameters(), lr=0.1)
        return [opt], [torch.optim.lr_scheduler.StepLR(opt, step_size=1)]

    def _loader(self):
        return DataLoader(RandomDataset(_IN, _LEN))

    def train_dataloader(self):
        return self._loader()

    def val_dataloader(self):
        return self._loader()

    def test_dataloader(self):
        return self._loader()

    # ---------------------------------------------------------- checkpoint
    def on_save_checkpoint(self, checkpoint):
        checkpoint["val_epoch"] = self.val_epoch

    def on_load_checkpoint(self, checkpoint) -> None:
        self.val_epoch = checkpoint["val_epoch"]
