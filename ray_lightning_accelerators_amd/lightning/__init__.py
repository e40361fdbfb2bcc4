"""PyTorch-Lightning-1.1-compatible surface (Trainer, LightningModule, callbacks, metrics).

``import ray_lightning_accelerators_amd.lightning as pl`` gives the names the
reference's tests and examples use: ``pl.Trainer``,
``pl.LightningModule``, ``pl.LightningDataModule``, ``pl.Callback``,
``pl.seed_everything``, ``pl.metrics.Accuracy``, ``pl.callbacks.EarlyStopping``.
"""
from . import metrics  # noqa: F401
from .accelerators import Accelerator, DataParallelAccelerator, DDPAccelerator  # noqa: F401
from .callbacks import Callback, EarlyStopping, LearningRateMonitor, ModelCheckpoint  # noqa: F401
from .core import LightningDataModule, LightningModule  # noqa: F401
from .loggers import CSVLogger  # noqa: F401
from .trainer import Trainer  # noqa: F401
from .utilities import atomic_save, seed_everything  # noqa: F401

__version__ = "1.1.7-rla"


class callbacks:  # noqa: N801 - `pl.callbacks.EarlyStopping` style access
    Callback = Callback
    EarlyStopping = EarlyStopping
    ModelCheckpoint = ModelCheckpoint
    LearningRateMonitor = LearningRateMonitor
