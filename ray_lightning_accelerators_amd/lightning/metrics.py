"""Stateful metrics (``pl.metrics.Accuracy``, reference tests/utils.py:143).

``compute()`` all-reduces the ``correct``/``total`` counters when a process
group is up.  The counters stay on the predictions' device:
``update`` never synchronises with the GPU."""
from __future__ import annotations

import torch
import torch.distributed as dist


class Metric:
    def __init__(self, compute_on_step: bool = True, dist_sync_on_step: bool = False):
        self.compute_on_step = compute_on_step
        self.dist_sync_on_step = dist_sync_on_step

    def __call__(self, *args, **kwargs):
        """PL 1.1 ``forward``: accumulate state AND return the value on this batch only."""
        if not self.compute_on_step:
            self.update(*args, **kwargs)
            return None
        saved = self._snapshot()
        self.reset()
        self.update(*args, **kwargs)
        batch_val = self._compute_local()
        self._merge(saved)
        return batch_val


class Accuracy(Metric):
    def __init__(self, threshold: float = 0.5, compute_on_step: bool = True, **kw):
        super().__init__(compute_on_step)
        self.threshold = threshold
        self.reset()

    def reset(self) -> None:
        # the counters live on the device of the first update (no host sync per batch)
        self.correct = torch.tensor(0.0)
        self.total = torch.tensor(0.0)

    def update(self, preds: torch.Tensor, target: torch.Tensor) -> None:
        preds = preds.detach()
        target = target.detach().to(preds.device)
        if preds.dim() == target.dim() + 1:
            pred_lbl = preds.argmax(dim=-1)
        elif preds.is_floating_point():
            pred_lbl = (preds >= self.threshold).long()
        else:
            pred_lbl = preds
        if self.correct.device != preds.device:
            self.correct = self.correct.to(preds.device)
            self.total = self.total.to(preds.device)
        self.correct = self.correct + (pred_lbl == target).sum().float()
        self.total = self.total + float(target.numel())

    def _snapshot(self):
        return (self.correct.clone(), self.total.clone())

    def _merge(self, saved) -> None:
        self.correct = self.correct + saved[0].to(self.correct.device)
        self.total = self.total + saved[1].to(self.total.device)

    def _compute_local(self) -> torch.Tensor:
        return self.correct / self.total.clamp(min=1.0)

    def compute(self) -> torch.Tensor:
        c, t = self.correct.clone(), self.total.clone()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dev = c.device
            buf = torch.stack([c, t])
            if dist.get_backend() == "nccl":
                buf = buf.cuda()
            elif buf.is_cuda:
                buf = buf.cpu()  # gloo takes host tensors
            dist.all_reduce(buf)
            c, t = buf[0].to(dev), buf[1].to(dev)
        return c / t.clamp(min=1.0)
