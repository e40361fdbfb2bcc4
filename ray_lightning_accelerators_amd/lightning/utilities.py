"""Small utilities of the Lightning-compatible layer: seeding, atomic save,
rank-zero helpers, logging.  (Reference call sites: PL_GLOBAL_SEED propagation
ray_ddp.py:154-159; atomic_save tune.py:5,133 of the reference.)"""
from __future__ import annotations

import logging
import os
import random
import tempfile
from functools import wraps
from typing import Any, Optional

import numpy as np
import torch

log = logging.getLogger("ray_lightning_accelerators_amd")
if not log.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("%(levelname)s %(name)s: %(message)s"))
    log.addHandler(_h)
    log.setLevel(logging.WARNING)


def seed_everything(seed: Optional[int] = None, workers: bool = False) -> int:
    """Seed python, numpy and torch; exported as ``PL_GLOBAL_SEED`` so the
    accelerators can forward it to their workers (reference ray_ddp.py:154-159)."""
    if seed is None:
        env = os.environ.get("PL_GLOBAL_SEED")
        seed = int(env) if env is not None else random.randint(0, 2 ** 31 - 1)
    seed = int(seed)
    os.environ["PL_GLOBAL_SEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    if workers:
        os.environ["PL_SEED_WORKERS"] = "1"
    return seed


def reset_seed() -> None:
    seed = os.environ.get("PL_GLOBAL_SEED")
    if seed is not None:
        seed_everything(int(seed))


def atomic_save(checkpoint: Any, filepath: str) -> None:
    """torch.save to a temp file in the same directory, then rename (atomic on POSIX)."""
    d = os.path.dirname(os.path.abspath(filepath)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp_ckpt_", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(checkpoint, f)
        os.replace(tmp, filepath)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def load_checkpoint(path: str, map_location: Any = "cpu") -> dict:
    """Load a Lightning checkpoint.  Files written by this framework contain
    only tensors/containers/primitives, so the safe ``weights_only`` loader is
    tried first; hparams objects of user classes fall back to a full load of
    OUR OWN files only (never used on third-party files)."""
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except Exception:
        return torch.load(path, map_location=map_location, weights_only=False)


class _RankZero:
    rank = 0


rank_zero_only_state = _RankZero()


def rank_zero_only(fn):
    @wraps(fn)
    def wrapped(*args, **kwargs):
        if rank_zero_only_state.rank == 0:
            return fn(*args, **kwargs)
        return None

    wrapped.rank = 0
    return wrapped


@rank_zero_only
def rank_zero_warn(msg: str) -> None:
    log.warning(msg)


@rank_zero_only
def rank_zero_info(msg: str) -> None:
    log.info(msg)


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def move_to_device(batch: Any, device: torch.device, non_blocking: bool = True) -> Any:
    if isinstance(batch, torch.Tensor):
        return batch.to(device, non_blocking=non_blocking)
    if isinstance(batch, (list, tuple)):
        out = [move_to_device(b, device, non_blocking) for b in batch]
        return type(batch)(out) if not hasattr(batch, "_fields") else type(batch)(*out)
    if isinstance(batch, dict):
        return {k: move_to_device(v, device, non_blocking) for k, v in batch.items()}
    return batch


def to_float(v: Any) -> float:
    if isinstance(v, torch.Tensor):
        return float(v.detach().float().mean().item())
    return float(v)
