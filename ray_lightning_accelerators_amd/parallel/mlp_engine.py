"""Data-parallel training engine for the MNIST classifier on the fused HIP step.

This is the worker-side hot loop that ``RayAccelerator`` / ``HorovodRayAccelerator``
run for ``MNISTClassifier`` (SURVEY.md §3.5 "one training step"), re-designed
for MI355X instead of translating PL's DDP loop:

* the dataset is resident in HBM as uint8 (MNIST is uint8; ToTensor's /255 is
  fused into the kernel), and each rank's DistributedSampler shard for the
  epoch is an index list on the device, so a step needs NO host->device copy;
* parameters, gradients and Adam state are flat fp32 arenas; the whole model's
  gradient is ONE allreduce bucket (27,882 floats = 109 KiB at the default
  32/64 config -- far below the ~1 MiB where splitting pays on 7 xGMI links);
* world size 1: ONE kernel launch per step (Adam fused into the gradient
  epilogues); world size > 1: fused fwd/bwd kernel -> allreduce(SUM) -> fused
  Adam with the 1/world average folded into ``grad_scale``;
* the step's device work can be captured into a hipGraph (``use_graph``): the
  batch cursor and step counter live on the device, so replays advance by
  themselves and the host only re-shuffles ``order`` at epoch boundaries.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist

from ..ops import fused_mlp
from ..ops.optim import fused_adam_


def shard_indices(n: int, world: int, rank: int, epoch: int, seed: int, shuffle: bool,
                  device=None) -> torch.Tensor:
    """torch.utils.data.DistributedSampler's index set for (rank, epoch)."""
    if shuffle:
        g = torch.Generator().manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g)
    else:
        idx = torch.arange(n)
    total = int(math.ceil(n / world)) * world
    if total > n:
        idx = torch.cat([idx, idx[: total - n]])
    out = idx[rank:total:world]
    return out.to(device) if device is not None else out


class FusedMLPEngine:
    def __init__(
        self,
        layer_1: int,
        layer_2: int,
        batch_size: int,
        lr: float = 1e-3,
        betas=(0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.0,
        device: Optional[torch.device] = None,
        world_size: int = 1,
        rank: int = 0,
        allreduce: Optional[Callable[[torch.Tensor], None]] = None,
        init_params: Optional[torch.Tensor] = None,
        stats_ring: int = 1024,
        seed: int = 0,
    ):
        if not fused_mlp.mlp_supported(layer_1, layer_2):
            raise ValueError(f"no fused kernel for layer sizes {layer_1}/{layer_2}")
        self.L1, self.L2, self.B = int(layer_1), int(layer_2), int(batch_size)
        self.lr, self.betas, self.eps, self.wd = float(lr), tuple(betas), float(eps), float(weight_decay)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.world_size, self.rank = int(world_size), int(rank)
        self.allreduce = allreduce
        n = fused_mlp.mlp_param_count(self.L1, self.L2)
        if init_params is None:
            init_params = fused_mlp.init_mlp_params(self.L1, self.L2, torch.Generator().manual_seed(seed))
        self.params = init_params.detach().to(self.device, torch.float32).contiguous().clone()
        self.grads = torch.zeros(n, device=self.device)
        self.exp_avg = torch.zeros(n, device=self.device)
        self.exp_avg_sq = torch.zeros(n, device=self.device)
        self.counters = torch.zeros(3, dtype=torch.int64, device=self.device)
        self.lr_tensor = torch.full((1,), self.lr, device=self.device)
        lay = fused_mlp.mlp_shadow_layout(self.L1, self.L2)
        self.shadow = torch.zeros(lay["total"], dtype=torch.bfloat16, device=self.device)
        self.dh1t = torch.zeros(self.L1 * ((self.B + 31) // 32 * 32), dtype=torch.bfloat16, device=self.device)
        self.kernel_version = 2
        self.refresh_shadow()
        self.stats = torch.zeros(stats_ring, 4, device=self.device)
        self.seed = seed
        self.epoch = 0
        self.step_in_epoch = 0
        self.global_step = 0
        self._graph = None
        self._graph_steps = 0
        self.x_u8 = self.labels = self.order = None
        self.n_batches = 0

    # ------------------------------------------------------------------ data
    def set_data(self, images_u8: torch.Tensor, labels: torch.Tensor, shuffle: bool = True) -> None:
        """Make the (full) dataset resident on the device; shards are per-rank index lists."""
        assert images_u8.dtype == torch.uint8 and images_u8.dim() == 2 and images_u8.size(1) == 784
        self.x_u8 = images_u8.to(self.device).contiguous()
        self.labels = labels.to(self.device, torch.int64).contiguous()
        self.shuffle = shuffle
        self.n_data = self.x_u8.size(0)
        per_rank = int(math.ceil(self.n_data / self.world_size))
        self.n_batches = per_rank // self.B
        if self.n_batches < 1:
            raise ValueError("dataset shard smaller than one batch")
        self.order = torch.empty(self.n_batches * self.B, dtype=torch.int64, device=self.device)
        self._load_epoch(0)

    def _load_epoch(self, epoch: int) -> None:
        idx = shard_indices(self.n_data, self.world_size, self.rank, epoch, self.seed, self.shuffle)
        idx = idx[: self.n_batches * self.B]
        assert int(idx.max()) < self.n_data and int(idx.min()) >= 0  # kernel trusts indices
        self.order.copy_(idx.to(self.device), non_blocking=True)
        self.epoch = epoch
        self.step_in_epoch = 0

    # ------------------------------------------------------------ broadcast
    def broadcast_from(self, src: int = 0) -> None:
        if self.world_size > 1 and dist.is_initialized():
            dist.broadcast(self.params, src)
        self.refresh_shadow()

    def refresh_shadow(self) -> None:
        """Rebuild the bf16 weight shadows after the fp32 params changed outside a step."""
        fused_mlp.mlp_refresh_shadow(self.params, self.shadow, self.L1, self.L2)

    def set_lr(self, lr: float) -> None:
        self.lr = float(lr)
        self.lr_tensor.fill_(self.lr)

    # ----------------------------------------------------------------- step
    def _device_step(self) -> None:
        fused = self.world_size == 1
        if self.kernel_version == 1:
            fused_mlp.mlp_train_step(
                self.params, self.grads, L1=self.L1, L2=self.L2, B=self.B, labels=self.labels,
                x_u8=self.x_u8, order=self.order, counters=self.counters[:2], n_batches=self.n_batches,
                exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq, stats=self.stats,
                apply_adam=fused, advance_step=True, lr=self.lr, betas=self.betas, eps=self.eps,
                weight_decay=self.wd, lr_tensor=self.lr_tensor,
            )
        else:
            fused_mlp.mlp_train_step2(
                self.params, self.grads, shadow=self.shadow, dh1t=self.dh1t, counters=self.counters, L1=self.L1,
                L2=self.L2, B=self.B, labels=self.labels, x_u8=self.x_u8, order=self.order,
                n_batches=self.n_batches, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq, stats=self.stats,
                apply_adam=fused, advance_step=True, lr=self.lr, betas=self.betas, eps=self.eps,
                weight_decay=self.wd, lr_tensor=self.lr_tensor,
            )
        if not fused:
            if self.allreduce is not None:
                self.allreduce(self.grads)
            if self.kernel_version == 1:
                fused_adam_(self.params, self.grads, self.exp_avg, self.exp_avg_sq, lr=self.lr,
                            betas=self.betas, eps=self.eps, weight_decay=self.wd,
                            grad_scale=1.0 / self.world_size, step=self.counters[0:1],
                            lr_tensor=self.lr_tensor)
            else:
                fused_mlp.mlp_adam_(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.shadow, L1=self.L1,
                                    L2=self.L2, lr=self.lr, step=self.counters[0:1], betas=self.betas, eps=self.eps,
                                    weight_decay=self.wd, grad_scale=1.0 / self.world_size,
                                    lr_tensor=self.lr_tensor)

    def _advance_host(self, n: int) -> None:
        self.global_step += n
        self.step_in_epoch += n
        if self.step_in_epoch >= self.n_batches:
            # the device cursor wrapped to 0 in the same step; load the next shuffle
            self._load_epoch(self.epoch + 1)

    def steps_to_epoch_end(self) -> int:
        return self.n_batches - self.step_in_epoch

    def capture(self, steps_per_graph: int = 1) -> bool:
        """Capture ``steps_per_graph`` consecutive steps into one hipGraph."""
        if self.device.type != "cuda":
            return False
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        # warm the allocator / RCCL outside capture (does a real step; keep counters consistent)
        with torch.cuda.stream(s):
            self._device_step()
        torch.cuda.current_stream().wait_stream(s)
        self._advance_host(1)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, stream=s):
                for _ in range(steps_per_graph):
                    self._device_step()
        except Exception:
            self._graph = None
            return False
        self._graph = g
        self._graph_steps = steps_per_graph
        return True

    def step(self) -> None:
        """Run one (or ``steps_per_graph`` when captured) optimizer step(s)."""
        if self._graph is not None and self.step_in_epoch + self._graph_steps <= self.n_batches:
            self._graph.replay()
            self._advance_host(self._graph_steps)
            return
        self._device_step()
        self._advance_host(1)

    def run(self, n_steps: int) -> None:
        done = 0
        while done < n_steps:
            k = self._graph_steps if self._graph is not None else 1
            if self._graph is not None and (n_steps - done < k or self.step_in_epoch + k > self.n_batches):
                self._device_step()
                self._advance_host(1)
                done += 1
                continue
            self.step()
            done += k

    # --------------------------------------------------------------- export
    def recent_stats(self, n: int = 1) -> torch.Tensor:
        """Last n (loss, correct, count, step) rows, oldest first (host copy)."""
        t = self.global_step
        ring = self.stats.size(0)
        rows = [(t - 1 - i) % ring for i in range(min(n, t, ring))][::-1]
        return self.stats[rows].cpu() if rows else torch.zeros(0, 4)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().cpu().clone() for k, v in fused_mlp.mlp_unpack(self.params, self.L1, self.L2).items()}

    def optimizer_state_dict(self) -> Dict:
        """torch.optim.Adam.state_dict() layout (Lightning checkpoint `optimizer_states`)."""
        step = float(self.counters[0].item())
        m = fused_mlp.mlp_unpack(self.exp_avg, self.L1, self.L2)
        v = fused_mlp.mlp_unpack(self.exp_avg_sq, self.L1, self.L2)
        state = {}
        for i, k in enumerate(m):
            state[i] = {"step": torch.tensor(step), "exp_avg": m[k].detach().cpu().clone(),
                        "exp_avg_sq": v[k].detach().cpu().clone()}
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "params": list(range(len(m)))}
        return {"state": state, "param_groups": [group]}
