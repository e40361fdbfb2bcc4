"""``MNISTDataModule`` (the pl_bolts data module the reference tests use,
tests/test_ddp.py:3,106-109) backed by synthetic MNIST-shaped data."""
from __future__ import annotations

from typing import Optional

import torch
from torch.utils.data import DataLoader, random_split

from ..lightning import LightningDataModule
from .data import SyntheticMNIST


class MNISTDataModule(LightningDataModule):
    name = "mnist"

    def __init__(self, data_dir: Optional[str] = None, val_split: int = 5000, num_workers: int = 0,
                 normalize: bool = False, batch_size: int = 32, seed: int = 42, n_train: int = 60000,
                 n_test: int = 10000, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.dims = (1, 28, 28)
        self.data_dir = data_dir
        self.val_split = val_split
        # worker subprocesses would fork a GPU-initialised process; data is in memory anyway
        self.num_workers = 0
        self.normalize = normalize
        self.batch_size = batch_size
        self.seed = seed
        self.n_train = n_train
        self.n_test = n_test
        self._train = self._val = self._test = None

    @property
    def num_classes(self) -> int:
        return 10

    def prepare_data(self, *args, **kwargs) -> None:
        pass  # nothing to download

    def setup(self, stage: Optional[str] = None) -> None:
        if stage in (None, "fit") and self._train is None:
            full = SyntheticMNIST(self.n_train, seed=0, train=True)
            self._train, self._val = random_split(
                full, [self.n_train - self.val_split, self.val_split],
                generator=torch.Generator().manual_seed(self.seed))
        if stage in (None, "test") and self._test is None:
            self._test = SyntheticMNIST(self.n_test, seed=0, train=False)

    def train_dataloader(self):
        self.setup("fit")
        return DataLoader(self._train, batch_size=self.batch_size, shuffle=True, num_workers=self.num_workers,
                          drop_last=True)

    def val_dataloader(self):
        self.setup("fit")
        return DataLoader(self._val, batch_size=self.batch_size, shuffle=False, num_workers=self.num_workers,
                          drop_last=True)

    def test_dataloader(self):
        self.setup("test")
        return DataLoader(self._test, batch_size=self.batch_size, shuffle=False, num_workers=self.num_workers,
                          drop_last=False)
