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


def _private_copy(obj: Any) -> Any:
    """The checkpoint dict with every tensor cloned, so a background write never
    reads storage the training loop keeps mutating (``.cpu()`` of a CPU tensor is
    the tensor itself)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().clone()
    if isinstance(obj, dict):  # dict / OrderedDict (state dicts)
        return type(obj)((k, _private_copy(v)) for k, v in obj.items())
    if type(obj) in (list, tuple):
        return type(obj)(_private_copy(v) for v in obj)
    return obj


class CheckpointWriter:
    """One background thread that runs checkpoint file operations in submission
    order (writes and the top-k removals that must follow them), so the epoch-end
    checkpoint write (~1.7 ms for the MNIST model: pickling + file I/O) overlaps
    the next epoch's GPU work instead of stalling it.  ``wait()`` drains the
    queue and re-raises the first error; the Trainer waits before ``fit``
    returns and before any synchronous save."""

    def __init__(self):
        import queue
        import threading

        self._q: "queue.Queue" = queue.Queue()
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._loop, name="rla-ckpt-writer", daemon=True)
        self._t.start()

    def _loop(self) -> None:
        while True:
            item = self._q.get()
            try:
                if item is None:
                    return
                fn, args = item
                if self._err is None:
                    fn(*args)
            except BaseException as e:  # noqa: BLE001 - surfaced by wait()
                self._err = e
            finally:
                self._q.task_done()

    def submit(self, fn, *args) -> None:
        self._raise()
        self._q.put((fn, args))

    def save(self, checkpoint: Any, filepath: str) -> None:
        self.submit(atomic_save, _private_copy(checkpoint), filepath)

    def wait(self) -> None:
        self._q.join()
        self._raise()

    def _raise(self) -> None:
        if self._err is not None:
            e, self._err = self._err, None
            raise RuntimeError(f"background checkpoint write failed: {e!r}") from e

    def close(self) -> None:
        self.wait()
        self._q.put(None)
        self._t.join(timeout=10)


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
