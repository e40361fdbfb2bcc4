"""Synthetic, MNIST-shaped data (no downloads are possible on this platform).

``synthetic_mnist`` produces uint8 28x28 images of a *learnable* 10-class task
(class-conditional stroke prototypes + per-sample jitter and noise), so the
reference's accuracy gates (>= 0.5 after 10 train batches,
ray_lightning/tests/utils.py:137-152 of the reference) remain meaningful.
Images are uint8 like real MNIST; the ``ToTensor`` scaling (x / 255) happens
in the dataset's ``__getitem__`` on CPU or inside the fused kernel on GPU.
"""
from __future__ import annotations

import math
import os
import tempfile
from typing import Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

IMG = 28


def _prototypes(seed: int = 0) -> torch.Tensor:
    """Ten class prototypes: two gaussian blobs per class on distinct ring angles."""
    yy, xx = torch.meshgrid(torch.arange(IMG).float(), torch.arange(IMG).float(), indexing="ij")
    protos = torch.zeros(10, IMG, IMG)
    for c in range(10):
        for k, r, s in ((c, 8.0, 2.5), ((3 * c + 1) % 10, 4.0, 2.0)):
            a = 2 * math.pi * k / 10
            cy, cx = 13.5 + r * math.sin(a), 13.5 + r * math.cos(a)
            protos[c] += torch.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        protos[c] /= protos[c].max()
    return protos


_CACHE_VERSION = 1
_memo = {}


def _cache_dir() -> str:
    return os.environ.get("RLA_DATA_CACHE") or os.path.join(tempfile.gettempdir(), "rla-synthetic-mnist")


def synthetic_mnist(n: int, seed: int = 0, noise: float = 0.1, jitter: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Return (images uint8 [n, 784], labels int64 [n]).

    Generated once per machine: the arrays are cached as ``.npy`` files (the
    stand-in for the reference's MNIST download into ``data_dir``), so every
    later Tune trial / training worker loads 47 MB in tens of milliseconds
    instead of regenerating it (~2.5 s single-threaded, which dominated the
    start-up of short trials).  ``RLA_DATA_CACHE=0`` disables the disk cache."""
    key = (n, seed, float(noise), jitter)
    if key in _memo:
        x, y = _memo[key]
        return x.clone(), y.clone()
    use_disk = os.environ.get("RLA_DATA_CACHE", "") != "0"
    stem = os.path.join(_cache_dir(), f"v{_CACHE_VERSION}_n{n}_s{seed}_z{noise:g}_j{jitter}")
    if use_disk:
        try:
            x = torch.from_numpy(np.load(stem + "_x.npy"))
            y = torch.from_numpy(np.load(stem + "_y.npy"))
            if x.shape == (n, IMG * IMG) and y.shape == (n,):
                _memo[key] = (x, y)
                return x.clone(), y.clone()
        except (OSError, ValueError):
            pass
    x, y = _generate(n, seed, noise, jitter)
    _memo[key] = (x, y)
    if use_disk:
        try:  # atomic publish: concurrent trials may race to write the same arrays
            os.makedirs(_cache_dir(), exist_ok=True)
            for suffix, arr in (("_x.npy", x), ("_y.npy", y)):
                tmp = f"{stem}{suffix}.{os.getpid()}.tmp"
                with open(tmp, "wb") as f:
                    np.save(f, arr.numpy())
                os.replace(tmp, stem + suffix)
        except OSError:
            pass
    return x.clone(), y.clone()


def _generate(n: int, seed: int, noise: float, jitter: int) -> Tuple[torch.Tensor, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    protos = _prototypes(0)  # class definitions are shared by every split
    labels = torch.randint(0, 10, (n,), generator=g)
    shifts = torch.randint(-jitter, jitter + 1, (n, 2), generator=g)
    imgs = protos[labels]
    # per-sample translation jitter (rolled in blocks of equal shift for speed)
    out = torch.empty(n, IMG, IMG)
    for dy in range(-jitter, jitter + 1):
        for dx in range(-jitter, jitter + 1):
            m = (shifts[:, 0] == dy) & (shifts[:, 1] == dx)
            if m.any():
                out[m] = torch.roll(imgs[m], shifts=(dy, dx), dims=(1, 2))
    out = out * (0.7 + 0.6 * torch.rand(n, 1, 1, generator=g)) + noise * torch.rand(n, IMG, IMG, generator=g)
    return (out.clamp(0, 1) * 255).round().to(torch.uint8).reshape(n, IMG * IMG), labels


class SyntheticMNIST(Dataset):
    """Map-style dataset yielding (float [1,28,28] in [0,1], label) like torchvision MNIST+ToTensor."""

    def __init__(self, n: int = 60000, seed: int = 0, train: bool = True):
        self.images, self.targets = synthetic_mnist(n, seed=seed if train else seed + 1)

    def __len__(self) -> int:
        return self.targets.numel()

    def __getitem__(self, i):
        return self.images[i].view(1, IMG, IMG).float() / 255.0, int(self.targets[i])


class RandomDataset(Dataset):
    """Gaussian vectors (reference tests/utils.py:12-21)."""

    def __init__(self, size: int, length: int, generator: Optional[torch.Generator] = None):
        self.len = length
        self.data = torch.randn(length, size, generator=generator)

    def __getitem__(self, index: int):
        return self.data[index]

    def __len__(self) -> int:
        return self.len
