"""Minimal experiment loggers: CSV (always available) with the Lightning
``lightning_logs/version_N`` directory convention."""
from __future__ import annotations

import csv
import os
from typing import Any, Dict, Optional

import torch


class LightningLoggerBase:
    def log_metrics(self, metrics: Dict[str, Any], step: Optional[int] = None) -> None:
        pass

    def log_hyperparams(self, params: Dict[str, Any]) -> None:
        pass

    def save(self) -> None:
        pass

    def finalize(self, status: str) -> None:
        self.save()

    @property
    def log_dir(self) -> Optional[str]:
        return None


class CSVLogger(LightningLoggerBase):
    NAME_METRICS_FILE = "metrics.csv"

    def __init__(self, save_dir: str, name: str = "lightning_logs", version: Optional[int] = None):
        self.save_dir = save_dir
        self.name = name
        self._version = version
        self._rows = []
        self._keys = []
        self.rank = 0

    @property
    def root_dir(self) -> str:
        return os.path.join(self.save_dir, self.name)

    @property
    def version(self) -> int:
        if self._version is None:
            self._version = self._next_version()
        return self._version

    def _next_version(self) -> int:
        root = self.root_dir
        if not os.path.isdir(root):
            return 0
        vs = []
        for d in os.listdir(root):
            if d.startswith("version_") and os.path.isdir(os.path.join(root, d)):
                try:
                    vs.append(int(d.split("_")[1]))
                except ValueError:
                    pass
        return max(vs) + 1 if vs else 0

    @property
    def log_dir(self) -> str:
        return os.path.join(self.root_dir, f"version_{self.version}")

    def log_metrics(self, metrics: Dict[str, Any], step: Optional[int] = None) -> None:
        if self.rank != 0:
            return
        row = {k: ((float(v) if v.numel() == 1 else float(v.detach().float().mean()))
                   if isinstance(v, torch.Tensor) else v) for k, v in metrics.items()}
        row["step"] = step
        for k in row:
            if k not in self._keys:
                self._keys.append(k)
        self._rows.append(row)

    def log_hyperparams(self, params: Dict[str, Any]) -> None:
        if self.rank != 0:
            return
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, "hparams.yaml"), "w") as f:
            for k, v in dict(params).items():
                f.write(f"{k}: {v!r}\n")

    def save(self) -> None:
        if self.rank != 0 or not self._rows:
            return
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, self.NAME_METRICS_FILE), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self._keys)
            w.writeheader()
            w.writerows(self._rows)
