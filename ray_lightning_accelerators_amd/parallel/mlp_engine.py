"""Data-parallel training engine for the MNIST classifier on the fused HIP step.

This is the worker-side hot loop that ``RayAccelerator`` / ``HorovodRayAccelerator``
run for ``MNISTClassifier`` (SURVEY.md §3.5 "one training step"; reference
``ray_lightning/tests/utils.py`` / ``examples/ray_ddp_example.py`` model),
re-designed for MI355X instead of translating PL's DDP loop:

* the dataset is resident in HBM as uint8 (MNIST is uint8; ToTensor's /255 is
  fused into the kernel), and each rank's DistributedSampler shard for the
  current AND the next epoch is an index list on the device, so a step needs
  NO host->device copy and no host sync at epoch boundaries;
* parameters, gradients and Adam state are flat fp32 arenas; the whole model's
  gradient is ONE allreduce bucket (27,882 floats = 109 KiB at the default
  32/64 config -- far below the ~1 MiB where splitting pays on 7 xGMI links);
* world size 1: ONE launch per step for B <= 32 (csrc/mlp_step3.hip kind Step1:
  every block replays the serial head chain on its own CU, then does its tail
  share), else TWO (head + 49-workgroup tail; Adam fused into both, the next
  step's layer 1 computed by the tail);
  world size > 1: with a ``dp_context`` the same launches, each block exchanging
  its gradient values with the peers over xGMI inside its Adam epilogue (kinds
  Step1DP / StepDP); otherwise head -> tail(grad) -> allreduce(SUM) ->
  tail(adam), the 1/world average folded into ``grad_scale``;
* the step's device work can be captured into a hipGraph (``capture``): batch
  cursor, step counter, ring slot and epoch buffer live on the device, so
  replays advance by themselves.

On a CPU device the same engine runs the fp32 PyTorch reference step (the
oracle of the GPU tests) with identical batch order and optimizer semantics.
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, Optional, Sequence

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
        buffers: Optional[Dict[str, torch.Tensor]] = None,
        dp_context: Optional[Sequence[int]] = None,
        dp_proto: Optional[str] = None,
        dp_rearm: Optional[Callable[[], None]] = None,
        dp_loop: bool = False,
    ):
        """``buffers``: optional external fp32 tensors ``params`` / ``grads`` /
        ``exp_avg`` / ``exp_avg_sq`` (e.g. views of a Trainer's parameter arena,
        so the nn.Module parameters stay the engine's master weights).
        ``dp_context``: ``NativeCommunicator.dp_context(...)`` -- world size > 1
        then runs the fused data-parallel step (the tail kernel exchanges its
        gradient tiles with the peers over xGMI inside the Adam epilogue: two
        launches per step, no separate allreduce).  ``dp_proto``: the one-launch
        step's exchange -- "packed" (one-shot, default), "owner" (reduce-scatter to
        the task's owner, Adam there, all-gather of the weights) or "granule" (round
        2); unset: ``RLA_DP_PROTO``.  ``dp_rearm``: collective reset of the exchange
        region (``NativeCommunicator.dp_rearm``), run before a protocol is first used.
        ``dp_loop``: loopback diagnostic (``dp_context`` of one process whose regions
        all point at its own; see scripts/dp_overhead_probe.py)."""
        if not fused_mlp.mlp_supported(layer_1, layer_2):
            raise ValueError(f"no fused kernel for layer sizes {layer_1}/{layer_2}")
        if not 1 <= batch_size <= 256:
            raise ValueError("fused MLP engine supports batch sizes 1..256")
        self.L1, self.L2, self.B = int(layer_1), int(layer_2), int(batch_size)
        self.lr, self.betas, self.eps, self.wd = float(lr), tuple(betas), float(eps), float(weight_decay)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.native = self.device.type == "cuda"
        self.world_size, self.rank = int(world_size), int(rank)
        self.allreduce = allreduce
        self.dp_ctx = None
        self.dp_loop = bool(dp_loop)
        if dp_context is not None and (self.world_size > 1 or self.dp_loop) and self.device.type == "cuda":
            ctx = [int(v) for v in dp_context]
            if not self.dp_loop and (ctx[0] != self.world_size or ctx[1] != self.rank):
                raise ValueError("dp_context belongs to a different (world, rank)")
            self.dp_ctx = ctx
        self._dp_rearm = dp_rearm
        self._owner_masks = None
        n = fused_mlp.mlp_param_count(self.L1, self.L2)
        if buffers is not None:
            for k in ("params", "grads", "exp_avg", "exp_avg_sq"):
                t = buffers[k]
                assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n and t.device == self.device, k
                setattr(self, k, t)
        else:
            if init_params is None:
                init_params = fused_mlp.init_mlp_params(self.L1, self.L2, torch.Generator().manual_seed(seed))
            self.params = init_params.detach().to(self.device, torch.float32).contiguous().clone()
            # padded to 4 floats: the xGMI one-shot allreduce moves 16-byte vectors
            self._grads_padded = torch.zeros((n + 3) // 4 * 4, device=self.device)
            self.grads = self._grads_padded[:n]
            self.exp_avg = torch.zeros(n, device=self.device)
            self.exp_avg_sq = torch.zeros(n, device=self.device)
        self.lr_tensor = torch.full((1,), self.lr, device=self.device)
        lay = fused_mlp.mlp_shadow_layout(self.L1, self.L2)
        self.shadow = torch.zeros(lay["total"], dtype=torch.bfloat16, device=self.device)
        bufs = fused_mlp.mlp3_buffers(self.L1, self.L2, self.B, self.device)
        # counters: [0] optimizer step, [1] next batch cursor, [2] last consumed cursor,
        # [3] H1pre/X ring slot, [4] epoch buffer of `order` that [1] indexes
        self.counters = bufs["counters"]
        self.dh1t, self.xring, self.h1pre, self.act = bufs["dh1t"], bufs["xring"], bufs["h1pre"], bufs["act"]
        self.yring = bufs["yring"]
        self.head_part = bufs["head_part"]
        self.hand = bufs["hand"]
        # world size 1, B <= 32: the whole step as ONE launch at every width
        # (RLA_MLP_ONE_LAUNCH=0: head + tail).  Round 5 gated widths > 64 off after
        # intermittent fidelity failures in long GPU sessions; round 6's post-mortem
        # showed the step bitwise equal to the two-launch step from a fresh engine in
        # the failing session (docs/one_launch_investigation.md), so the gate is gone.
        self.one_launch = self.B <= fused_mlp.ONE_LAUNCH_MAX_B and os.environ.get("RLA_MLP_ONE_LAUNCH") != "0"
        # world size > 1 with the xGMI context: the same one launch, each block
        # exchanging its values with the peers (protocol: self.dp_proto)
        self.dp_proto = "packed"
        self.one_launch_dp = False
        # (collective with a rearm callable: every rank builds its engine together)
        self.set_dp_proto(dp_proto or os.environ.get("RLA_DP_PROTO") or "packed", rearm=True)
        self.stats = torch.zeros(stats_ring, 4, device=self.device)
        self.seed = seed
        self.epoch = 0
        self.step_in_epoch = 0
        self.global_step = 0
        self._graph = None
        self._graph_steps = 0
        self._tail_graphs: Dict[int, "torch.cuda.CUDAGraph"] = {}  # remainder sizes (powers of two)
        self._shadow_stale = False
        self._primed = False
        self._host_epochs = False
        self.x_u8 = self.labels = self.order = None
        self.n_batches = 0
        self.refresh_shadow()

    # ------------------------------------------------- exchange protocol
    def set_dp_proto(self, name: str, rearm: bool = True) -> None:
        """Select the one-launch step's exchange protocol ("packed" / "owner" /
        "granule"; "wave" / "all" are two-launch flag protocols).  Collective when
        ``rearm`` (every rank switches together): the region is reset first, because
        a granule left by another protocol could carry a current-looking tag."""
        n = fused_mlp.mlp_param_count(self.L1, self.L2)
        if name not in fused_mlp.DP_PROTOS and name not in ("wave", "all"):
            raise ValueError(f"unknown data-parallel exchange protocol {name!r}")
        if self.dp_proto == "owner" and name != "owner" and getattr(self, "_stepped_owner", False):
            # leaving owner: non-owners' Adam state is stale -- consolidate first
            self.sync_optimizer_state()
        self._stepped_owner = False
        self.dp_proto = name
        ctx = self.dp_ctx
        need = 2 * n if name == "granule" else fused_mlp.DP_AREA_FLOATS
        self.one_launch_dp = (self.one_launch and ctx is not None and name in fused_mlp.DP_PROTOS
                              and ctx[2] >= need)
        if rearm and self.dp_ctx is not None and self._dp_rearm is not None:
            self._dp_rearm()
        self._drop_graphs()

    def dp_owner_mask(self, rank: Optional[int] = None) -> torch.Tensor:
        """Bool mask over the parameter arena: the elements whose Adam state this rank
        keeps under the "owner" protocol (mirror of the kernel's dp_task_owner: W1
        tile kt -> task kt; dW2 tile (ct, nt) -> 49 + ct * (L2/16) + nt; dW3 tile nt ->
        49 + (L1/16)(L2/16) + nt; bias chunk of 64 -> after those; owner = task % N)."""
        rank = self.rank if rank is None else int(rank)
        world = self.dp_ctx[0] if self.dp_ctx is not None else self.world_size
        L1, L2 = self.L1, self.L2
        tn1, tn2 = L1 // 16, L2 // 16
        tiles = 784 // 16
        w1 = (torch.arange(784) // 16).repeat(L1)  # [L1 rows][784 pixels], row-major
        nb = L1 + L2 + 10
        w2 = tiles + (torch.arange(L1) // 16).repeat(L2) * tn2 + (torch.arange(L2) // 16).repeat_interleave(L1)
        w3 = tiles + tn1 * tn2 + (torch.arange(L2) // 16).repeat(10)
        bias = tiles + tn1 * tn2 + tn2 + torch.arange(nb) // 64
        b1, b2, b3 = bias[:L1], bias[L1:L1 + L2], bias[L1 + L2:]
        task = torch.cat([w1, b1, w2, b2, w3, b3])  # arena order: W1 B1 W2 B2 W3 B3
        assert task.numel() == fused_mlp.mlp_param_count(L1, L2)
        return (task % world) == rank

    def sync_optimizer_state(self) -> None:
        """Owner protocol: every rank's Adam state becomes the owners' (each element's
        current m / v live only on its task's owner) -- a masked SUM allreduce, exact
        (one nonzero term).  Collective; run before anything reads exp_avg /
        exp_avg_sq (checkpoints, optimizer_state_dict, a protocol switch)."""
        if not (self.native and self.one_launch_dp and self.dp_proto == "owner" and self.world_size > 1):
            return
        if self.dp_loop:
            return  # loopback: one process holds every "rank's" state
        if self.allreduce is None:
            raise RuntimeError("owner protocol: sync_optimizer_state needs the engine's allreduce")
        if self._owner_masks is None:
            self._owner_masks = self.dp_owner_mask().to(self.device, torch.float32)
        for t in (self.exp_avg, self.exp_avg_sq):
            t.mul_(self._owner_masks)
            self.allreduce(t)

    def _publish_counters(self) -> None:
        """Host edits of the device state go to both copies (current / advanced)."""
        self.counters[5:10].copy_(self.counters[0:5])

    def check(self, blocking: bool = True) -> None:
        """Raise if a one-launch step's in-launch hand-off ever timed out (a block
        polled past its bound: the step it belongs to is not trustworthy).
        ``blocking=False`` (the Trainer's epoch ends): the flag is copied to pinned
        host memory asynchronously and the copy made at the PREVIOUS call is the one
        checked -- no device sync at an epoch boundary, detection one epoch late; a
        blocking call at the end of the fit reads the current value."""
        if not self.native:
            return
        prev = getattr(self, "_hand_probe", None)
        if prev is not None:
            buf, ev = prev
            ev.synchronize()  # enqueued one epoch ago: long complete
            self._hand_probe = None
            if int(buf[0]) != 0:
                raise RuntimeError("fused MLP one-launch step: an in-launch hand-off timed out")
        if blocking:
            if int(self.hand[16].item()) != 0:
                raise RuntimeError("fused MLP one-launch step: an in-launch hand-off timed out")
            return
        buf = getattr(self, "_hand_pin", None)
        if buf is None:
            buf = self._hand_pin = torch.zeros(1, dtype=self.hand.dtype, pin_memory=True)
        buf.copy_(self.hand[16:17], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._hand_probe = (buf, ev)

    def set_step(self, step: int) -> None:
        self.counters[0] = int(step)
        self._publish_counters()

    @property
    def comm_buffer(self) -> torch.Tensor:
        """The gradient bucket handed to the allreduce (16-byte padded when owned)."""
        return getattr(self, "_grads_padded", self.grads)

    # ------------------------------------------------- host-driven epochs
    def attach_dataset(self, images_u8: torch.Tensor, labels: torch.Tensor) -> None:
        """Trainer mode: the dataset is resident, the host supplies each epoch's order."""
        assert images_u8.dtype == torch.uint8 and images_u8.dim() == 2 and images_u8.size(1) == 784
        self.x_u8 = images_u8.to(self.device).contiguous()
        self.labels = labels.to(self.device, torch.int64).contiguous()
        self.n_data = self.x_u8.size(0)
        self._host_epochs = True

    def begin_epoch(self, order: torch.Tensor, n_batches: int, checked: bool = False) -> None:
        """Load one epoch's sample order ([n_batches * B] indices) and re-prime.

        Both order buffers get the same list, so the last step's look-ahead
        gather wraps into valid indices; the next ``begin_epoch`` re-primes."""
        order = order.reshape(-1)[: n_batches * self.B]
        assert n_batches >= 1 and order.numel() == n_batches * self.B
        # the kernels trust indices (a host order is checked without a device sync;
        # ``checked``: the caller already did)
        if not checked or order.device.type != "cpu":
            assert int(order.max()) < self.n_data and int(order.min()) >= 0
        if self.order is None or self.order.size(1) != order.numel() or self.n_batches != int(n_batches):
            # the captured graph bakes the order pointer and n_batches: only a new
            # shape forces a re-capture, a new epoch of the same shape reuses it
            self.order = torch.empty(2, order.numel(), dtype=torch.int64, device=self.device)
            self._drop_graphs()
        if order.device.type == "cpu" and self.native:
            # staged through a pinned buffer: an async H2D copy instead of a blocking
            # pageable one; the previous epoch's copy must be done before reuse
            if getattr(self, "_order_ev", None) is not None:
                self._order_ev.synchronize()
            pin = getattr(self, "_order_pin", None)
            if pin is None or pin.numel() != order.numel():
                pin = self._order_pin = torch.empty(order.numel(), dtype=torch.int64, pin_memory=True)
            pin.copy_(order)
            self.order[0].copy_(pin, non_blocking=True)
            self._order_ev = torch.cuda.Event()
            self._order_ev.record()
        else:
            self.order[0].copy_(order.to(self.device))
        self.order[1].copy_(self.order[0])
        self.n_batches = int(n_batches)
        self.counters[1:5].zero_()
        self._publish_counters()
        self.step_in_epoch = 0
        self._primed = False

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
        self.order = torch.empty(2, self.n_batches * self.B, dtype=torch.int64, device=self.device)
        self._fill_order(0)
        self._fill_order(1)
        self.counters[1:5].zero_()
        self._publish_counters()
        self.epoch = 0
        self.step_in_epoch = 0
        self._drop_graphs()
        self._primed = False

    def _fill_order(self, epoch: int) -> None:
        """Write ``epoch``'s shard order into buffer ``epoch % 2`` (stream-ordered)."""
        idx = shard_indices(self.n_data, self.world_size, self.rank, epoch, self.seed, self.shuffle)
        idx = idx[: self.n_batches * self.B]
        assert int(idx.max()) < self.n_data and int(idx.min()) >= 0  # the kernels trust indices
        self.order[epoch % 2].copy_(idx.to(self.device), non_blocking=True)

    # ------------------------------------------------------------ broadcast
    def broadcast_from(self, src: int = 0) -> None:
        if self.world_size > 1 and dist.is_initialized():
            if self.params.is_cuda and dist.get_backend() == "gloo":  # CPU bootstrap group
                tmp = self.params.cpu()
                dist.broadcast(tmp, src)
                self.params.copy_(tmp)
            else:
                dist.broadcast(self.params, src)
        self.refresh_shadow()

    def refresh_shadow(self) -> None:
        """Rebuild the bf16 weight shadows after the fp32 params changed outside a step."""
        fused_mlp.mlp_refresh_shadow(self.params, self.shadow, self.L1, self.L2)
        self._shadow_stale = False
        self._primed = False

    def load_params(self, flat: torch.Tensor) -> None:
        with torch.no_grad():
            self.params.copy_(flat.reshape(-1).to(self.params))
        self.refresh_shadow()

    def set_lr(self, lr: float) -> None:
        self.lr = float(lr)
        self.lr_tensor.fill_(self.lr)

    # ----------------------------------------------------------------- step
    def _kw3(self) -> dict:
        return dict(x_u8=self.x_u8, labels=self.labels, order=self.order, counters=self.counters,
                    n_batches=self.n_batches, B=self.B, L1=self.L1, L2=self.L2, params=self.params,
                    grads=self.grads, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq, shadow=self.shadow,
                    dh1t=self.dh1t, xring=self.xring, h1pre=self.h1pre, act=self.act, yring=self.yring,
                    head_part=self.head_part, hand=self.hand, lr=self.lr, betas=self.betas,
                    eps=self.eps, weight_decay=self.wd, lr_tensor=self.lr_tensor)

    def prime(self) -> None:
        """Layer-1 pre-activations of the pending batch from the current weights."""
        if self._shadow_stale:
            self._shadow_stale = False
            fused_mlp.mlp_refresh_shadow(self.params, self.shadow, self.L1, self.L2)
        if self.native:
            self.h1pre.zero_()
            fused_mlp.mlp3_launch(fused_mlp.MLP3_PRIME, **self._kw3())
        self._primed = True

    def _device_step(self) -> None:
        """One optimizer step on the device (or the fp32 reference step on the CPU)."""
        if self.x_u8 is None:
            raise RuntimeError("set_data() first")
        if not self._primed:
            self.prime()
        if not self.native:
            self._reference_step()
        else:
            kw = self._kw3()
            if self.world_size == 1 and not self.dp_loop:
                kind = fused_mlp.MLP3_STEP1 if self.one_launch else fused_mlp.MLP3_STEP
                fused_mlp.mlp3_launch(kind, stats=self.stats, **kw)
            elif self.dp_ctx is not None:
                kind = fused_mlp.MLP3_STEP1_DP if self.one_launch_dp else fused_mlp.MLP3_STEP_DP
                fused_mlp.mlp3_launch(kind, stats=self.stats, grad_scale=1.0 / self.dp_ctx[0],
                                      dp_ctx=self.dp_ctx, dp_proto=fused_mlp.DP_PROTOS.get(self.dp_proto, -1),
                                      dp_loop=self.dp_loop, **kw)
                self._stepped_owner = self._stepped_owner or (self.one_launch_dp and self.dp_proto == "owner")
            else:
                fused_mlp.mlp3_launch(fused_mlp.MLP3_HEAD, stats=self.stats, **kw)
                fused_mlp.mlp3_launch(fused_mlp.MLP3_TAIL_GRAD, stats=self.stats, **kw)  # multi-block head stats
                if self.allreduce is not None:
                    self.allreduce(self.comm_buffer)
                fused_mlp.mlp3_launch(fused_mlp.MLP3_TAIL_ADAM, grad_scale=1.0 / self.world_size, **kw)

    def _reference_step(self) -> None:
        """fp32 PyTorch step with the device kernels' batch / counter semantics."""
        c = self.counters
        cursor, ob = int(c[1]), int(c[4])
        fused = self.world_size == 1
        fused_mlp.mlp_train_step(
            self.params, self.grads, L1=self.L1, L2=self.L2, B=self.B, labels=self.labels, x_u8=self.x_u8,
            order=self.order[ob], counters=c[:2], n_batches=self.n_batches, exp_avg=self.exp_avg,
            exp_avg_sq=self.exp_avg_sq, stats=self.stats, apply_adam=fused, advance_step=True, lr=self.lr,
            betas=self.betas, eps=self.eps, weight_decay=self.wd, lr_tensor=self.lr_tensor,
        )
        c[2] = cursor
        c[3] = int(c[3]) ^ 1
        if cursor + 1 >= self.n_batches:
            c[4] = ob ^ 1
        self._publish_counters()
        if not fused:
            if self.allreduce is not None:
                self.allreduce(self.comm_buffer)
            fused_adam_(self.params, self.grads, self.exp_avg, self.exp_avg_sq, lr=self.lr, betas=self.betas,
                        eps=self.eps, weight_decay=self.wd, grad_scale=1.0 / self.world_size,
                        step=self.counters[0:1], lr_tensor=self.lr_tensor)

    def _advance_host(self, n: int) -> None:
        self.global_step += n
        self.step_in_epoch += n
        if self.step_in_epoch >= self.n_batches:
            # the device switched to the other order buffer in the same step
            self.epoch += 1
            self.step_in_epoch = 0
            if self._host_epochs:
                return  # the host calls begin_epoch()
            # buffer (epoch + 1) % 2 was last read by the step just enqueued
            self._fill_order(self.epoch + 1)

    def steps_to_epoch_end(self) -> int:
        return self.n_batches - self.step_in_epoch

    def _drop_graphs(self) -> None:
        self._graph = None
        self._tail_graphs = {}

    def capture(self, steps_per_graph: int = 1, remainders: bool = True) -> bool:
        """Capture ``steps_per_graph`` consecutive steps into one hipGraph.

        ``remainders``: also capture 1, 2, 4, ... step graphs below it, so a
        dispatch that is not a multiple of ``steps_per_graph`` (the Trainer's
        chunks end at log / validation / epoch boundaries) runs as a few replays
        instead of eager launches (~40 us of host work per eager step against
        ~9 us of GPU time, so eager remainders starved the GPU)."""
        if not self.native:
            return False
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        # warm the allocator / RCCL outside capture (a real step; keeps counters consistent)
        with torch.cuda.stream(s):
            self._device_step()
        torch.cuda.current_stream().wait_stream(s)
        self._advance_host(1)

        def record(n: int):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    self._device_step()
            return g

        try:
            g = record(steps_per_graph)
        except Exception:
            self._drop_graphs()
            return False
        self._graph = g
        self._graph_steps = steps_per_graph
        self._tail_graphs = {}
        if remainders:
            k = 1
            while k < steps_per_graph:
                try:
                    self._tail_graphs[k] = record(k)  # capture only: the device state does not move
                except Exception:
                    break
                k *= 2
        return True

    def _graph_ok(self, remaining: int, k: Optional[int] = None) -> bool:
        k = self._graph_steps if k is None else k
        return (self._graph is not None and self._primed and remaining >= k
                and self.step_in_epoch + k <= self.n_batches)

    def _pick_graph(self, remaining: int):
        """The largest captured graph that fits the remaining steps (and the epoch)."""
        if self._graph_ok(remaining):
            return self._graph, self._graph_steps
        for k in sorted(self._tail_graphs, reverse=True):
            if self._graph_ok(remaining, k):
                return self._tail_graphs[k], k
        return None, 1

    def step(self) -> None:
        """Run one (or ``steps_per_graph`` when captured) optimizer step(s)."""
        if self._graph_ok(self._graph_steps):
            self._graph.replay()
            self._advance_host(self._graph_steps)
            return
        self._device_step()
        self._advance_host(1)

    def run(self, n_steps: int) -> None:
        done = 0
        while done < n_steps:
            g, k = self._pick_graph(n_steps - done)
            if g is not None:
                g.replay()
            else:
                self._device_step()
            self._advance_host(k)
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
        """torch.optim.Adam.state_dict() layout (Lightning checkpoint `optimizer_states`).
        Collective under the owner protocol (state consolidation)."""
        self.sync_optimizer_state()
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
