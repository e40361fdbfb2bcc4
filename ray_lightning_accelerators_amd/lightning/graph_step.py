"""Whole-step hipGraph capture for autograd LightningModules.

The reference's contract is that all training runs inside the worker's
``Trainer`` (``/root/reference/ray_lightning/ray_ddp.py:199-220``: ``ddp_train``
at ``:218-219``).  An eager autograd step of a large convolutional model issues
hundreds of kernels from Python -- ResNet-50 is ~600 launches and ~17 ms of host
work per step (``profiles/r3_wgrad/rn50_host.log``) against ~14 ms of GPU work,
so an eager Trainer would be host-bound.  ``GraphedTrainStep`` makes the
Trainer's own per-batch step (``training_step`` -> backward -> gradient
all-reduce -> optimizer step -> ``zero_grad``) one hipGraph replay:

  * **warm-up**: the first ``warmup`` steps run eagerly on a side stream through
    the same step body (allocator pools, MIOpen solver search, the convolution
    autotune of ``ops/conv.py``); the first one under a host-read probe (a
    ``TorchFunctionMode`` that records ``.item()`` / ``.cpu()`` / ``bool(t)`` ...
    issued by user code: such a step cannot be replayed);
  * **capture**: one step recorded into a ``torch.cuda.CUDAGraph``: forward,
    loss, backward, the ``GradSynchronizer`` buckets forked onto the comm
    engine's stream (xGMI generation counters / RCCL: nothing host-side per
    step), the fused arena optimizer reading its step counter and learning rate
    from device scalars (``parallel/fused_optim.py``), and the write of the
    step's logged scalars into a device ring;
  * **replay**: one graph launch per step.  The Python side of ``self.log`` is
    replayed from the ring (views, no host sync): ``callback_metrics``, the
    logger and ``training_epoch_end`` see every step's own values;
  * **data**: a device-resident dataset (``SyntheticImageNet`` / ``TensorDataset``,
    ``lightning/sampling.py``) is gathered INSIDE the graph from a per-epoch
    device copy of the ``DistributedSampler`` order and a device cursor (no
    loader, no H2D per step; the Trainer then dispatches many steps per host
    call).  Any other loader's batch is copied into static input buffers before
    the replay; a batch of another shape runs eagerly.

Anything the probe, the static checks or the capture itself rejects falls back
to the Trainer's eager path with the reason logged (``reason``).  Opt-in: a
module sets ``hip_graph_step = True`` (``LightningResNet50`` does), or
``RLAConfig.hip_graph_step`` / ``RLA_HIP_GRAPH_STEP`` is ``"on"``.
"""
from __future__ import annotations

import os
import sys
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch.overrides import TorchFunctionMode
from torch.utils._pytree import tree_flatten, tree_unflatten

from ..config import get_config
from .callbacks import Callback
from .core import LightningModule
from .sampling import gather_rows, loader_order, resident_tensors
from .utilities import log

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_TORCH_DIR = os.path.dirname(os.path.abspath(torch.__file__))

# tensor methods / functions whose result the host must wait for
_HOST_READS = {
    torch.Tensor.item, torch.Tensor.tolist, torch.Tensor.numpy, torch.Tensor.__bool__,
    torch.Tensor.__float__, torch.Tensor.__int__, torch.Tensor.__index__, torch.Tensor.cpu,
    torch.Tensor.nonzero, torch.nonzero, torch.masked_select, torch.Tensor.masked_select,
    torch.unique, torch.Tensor.unique, torch.Tensor.__repr__, torch.Tensor.__format__,
    torch.Tensor.any, torch.Tensor.all,
}


class HostReadProbe(TorchFunctionMode):
    """Record host reads of tensor values made by code outside this package and
    outside torch itself (the framework's own first-use autotuning syncs on
    purpose, and only during warm-up).  ``any`` / ``all`` count only when their
    result is converted on the host; they are listed so their callers are seen."""

    def __init__(self):
        super().__init__()
        self.reads: List[str] = []

    @staticmethod
    def _user_frame() -> Optional[str]:
        f = sys._getframe(2)
        while f is not None:
            fn = os.path.abspath(f.f_code.co_filename)
            if fn.startswith(_TORCH_DIR) or "torch/overrides" in fn:
                f = f.f_back
                continue
            if fn.startswith(_PKG_DIR) and not fn.startswith(os.path.join(_PKG_DIR, "models")):
                return None  # framework code (ops autotune, arena bookkeeping)
            return f"{fn}:{f.f_lineno}"
        return None

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        host = func in _HOST_READS and func not in (torch.Tensor.any, torch.Tensor.all)
        if not host and func is torch.Tensor.to:
            dev = kwargs.get("device", args[1] if len(args) > 1 else None)
            host = isinstance(dev, (str, torch.device)) and torch.device(dev).type == "cpu"
        if host:
            where = self._user_frame()
            if where is not None:
                self.reads.append(f"{getattr(func, '__name__', str(func))} at {where}")
        return func(*args, **kwargs)


def wanted(trainer, model) -> bool:
    """Whether the Trainer should try a graph-captured step for ``model``."""
    mode = str(get_config().hip_graph_step).lower()
    if mode == "off" or trainer.fused_step is False:
        return False
    attr = getattr(model, "hip_graph_step", None)
    if attr is False:
        return False
    return mode == "on" or attr is True


def static_reason(trainer, model) -> Optional[str]:
    """Why the step cannot be captured, judged before running it (None: try)."""
    opts = trainer.optimizers
    if len(opts) != 1:
        return f"{len(opts)} optimizers (one fused optimizer expected)"
    opt = opts[0]
    if not getattr(opt, "_rla_fused", False) or not hasattr(opt, "enable_device_scalars"):
        return f"optimizer {type(opt).__name__} is not fused onto the parameter arena"
    if trainer.accelerator_backend is None or getattr(trainer.accelerator_backend, "arena", None) is None:
        return "no parameter arena"
    if trainer.accumulate_grad_batches != 1:
        return "accumulate_grad_batches > 1"
    hst = getattr(opt, "_hvd_state", None)
    if hst is not None and trainer.world_size > 1:
        from ..horovod import Average, Compression

        if hst.op != Average or hst.compression is not Compression.none or hst.bpps != 1:
            return "Horovod DistributedOptimizer with op / compression / backward_passes_per_step other than the default"
    t = type(model)
    for name in ("backward", "optimizer_step", "optimizer_zero_grad", "on_after_backward", "on_before_zero_grad"):
        if getattr(t, name) is not getattr(LightningModule, name) or name in model.__dict__:
            return f"LightningModule.{name} is overridden (it would run once, at capture)"
    for cb in trainer.callbacks:
        for name in ("on_after_backward", "on_before_zero_grad"):
            fn = getattr(type(cb), name, None)
            if fn is not None and fn is not getattr(Callback, name):
                return f"callback {type(cb).__name__}.{name} (it would run once, at capture)"
    return None


class GraphedTrainStep:
    """The Trainer's autograd step as one hipGraph replay (module docstring).

    Implements the Trainer's fused-step protocol: ``train_batch`` (per batch),
    ``make_epoch_batches`` / ``train_chunk`` / ``log_points`` (resident data, many
    steps per dispatch), ``sync_params_to_module`` / ``load_params_from_module``."""

    chunk_spans_log_points = True
    counts_steps = True  # train_batch advances trainer.global_step itself

    def __init__(self, trainer, model, warmup: int = 3):
        self.trainer, self.model = trainer, model
        self.acc = trainer.accelerator_backend
        self.opt = trainer.optimizers[0]
        self.arena = self.acc.arena
        self.dev = self.arena.device
        self.cuda = self.dev.type == "cuda" and torch.cuda.is_available()
        self.warmup = max(1, int(warmup))
        self.reason: Optional[str] = None if self.cuda else "no GPU: the step body runs eagerly"
        self.failed = False  # the Trainer's eager autograd path runs every later step
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.steps_done = 0
        self.replays = 0
        self._log_meta: Optional[List[Tuple[str, str, dict]]] = None
        self._out_keys: Optional[List[str]] = None
        self._static: Optional[list] = None
        self._spec = None
        self._resident = None
        self._order: Optional[torch.Tensor] = None
        self._cursor: Optional[torch.Tensor] = None
        self._B = 0
        self._nb = 0
        self._last_rows = None
        self._last_batch = None
        self._eval_resident: Dict[int, Any] = {}
        self.opt.enable_device_scalars()
        if getattr(self.opt, "_hvd_state", None) is not None and trainer.world_size > 1:
            self._adopt_horovod()
        n = max(int(getattr(trainer, "num_training_batches", 0) or 0), 1)
        # two epochs of rows: an epoch's step outputs (ring views) stay valid through
        # its training_epoch_end and the next epoch's blocking log flush
        self.ring_rows = int(min(max(1024, 2 * n + 2), 1 << 20))
        self._ring: Optional[torch.Tensor] = None
        self._ring_pos = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._side = torch.cuda.Stream() if self.cuda else None

    def _adopt_horovod(self) -> None:
        """Horovod at world > 1: ``hvd.DistributedOptimizer``'s fusion engine negotiates
        and packs on a host thread, which no graph can record.  The same reduction --
        the averaged sum of every rank's gradient -- runs instead through the DDP
        ``GradSynchronizer`` (arena buckets, allreduce on the comm engine's stream,
        the 1/size average folded into the fused optimizer): the optimizer's fusion
        hooks are removed, ``synchronize()`` becomes the synchroniser's ``finish()``.
        Same math as ``op=Average``, capturable."""
        import types

        from ..parallel.ddp import GradSynchronizer

        st = self.opt._hvd_state
        for h in st.hooks:
            h.remove()
        st.hooks = []
        st.skip = True  # DistributedOptimizer.step no longer synchronises itself
        thr = float(os.environ.get("HOROVOD_FUSION_THRESHOLD", str(8 * 1024 * 1024))) / (1 << 20)
        sync = GradSynchronizer(self.model, self.arena, bucket_cap_mb=max(thr, 0.25), average_in_optimizer=True)
        self.acc.sync = sync  # before_forward / grad_scale of the accelerator use it
        self.opt.synchronize = types.MethodType(lambda _self: sync.finish(), self.opt)
        self.horovod_adopted = True

    # ------------------------------------------------------------ describe
    def describe(self) -> Dict[str, Any]:
        return {"captured": self.graph is not None, "replays": self.replays, "steps": self.steps_done,
                "fallback": self.reason if (self.failed or self.graph is None) else None,
                "resident_data": self._resident is not None, "warmup_steps": self.warmup}

    # ------------------------------------------------------------ step body
    def _body(self, batch_fn, batch_idx: int, probe: bool = False):
        """One training step exactly as ``Trainer._optimizer_step_for`` runs it, with
        every ``self.log`` recorded (not stored) and the step's scalars written to the
        ring row ``_ring_pos``.  Everything that can reject the step is checked
        before backward (a rejected step has not updated anything but BN running
        statistics, and is re-run by the eager path).  Returns (layout, values):
        ``layout`` = (log meta, output keys), ``values`` the recorded tensors."""
        t, model, acc, opt = self.trainer, self.model, self.acc, self.opt
        calls: List[tuple] = []
        batch = batch_fn()
        self._last_batch = batch  # a rejected resident step re-runs THIS batch eagerly
        # eager (not captured) step: the forward's buffer updates (BatchNorm running
        # statistics, num_batches_tracked) are undone if the step is rejected below,
        # so the eager re-run applies them once
        saved = None
        if not torch.cuda.is_available() or not torch.cuda.is_current_stream_capturing():
            saved = [(b, b.detach().clone()) for b in model.buffers()]
        try:
            return self._body_checked(t, model, acc, opt, calls, batch, batch_idx, probe)
        except _Unsupported:
            if saved is not None:
                with torch.no_grad():
                    for b, c in saved:
                        b.copy_(c)
            raise

    def _body_checked(self, t, model, acc, opt, calls, batch, batch_idx: int, probe: bool):
        acc.before_forward(sync=True)
        t._log_sink = calls
        mode = HostReadProbe() if probe else None
        try:
            if mode is not None:
                mode.__enter__()
            try:
                t._current_fx = "training_step"
                with acc.autocast():
                    out = model.training_step(batch, batch_idx)
                t._current_fx = "training_step_end"
                out = model.training_step_end(out)
            finally:
                if mode is not None:
                    mode.__exit__(None, None, None)
        finally:
            t._log_sink = None
            t._current_fx = None
        if out is None:
            raise _Unsupported("training_step returned None (skipped batch)")
        loss = out if isinstance(out, torch.Tensor) else out["loss"]
        extra = []
        if isinstance(out, dict):
            for k, v in out.items():
                if k == "loss":
                    continue
                if not (isinstance(v, torch.Tensor) and v.numel() == 1):
                    raise _Unsupported(f"training_step output {k!r} is not a scalar tensor")
                extra.append((k, v))
        for name, v, kw, _fx in calls:
            if kw.get("sync_dist"):
                raise _Unsupported(f"self.log({name!r}, sync_dist=True) (a host collective per step)")
            if not isinstance(v, torch.Tensor) or v.numel() != 1:
                raise _Unsupported(f"self.log({name!r}) of a non-scalar value")
        if mode is not None and mode.reads:
            self.reason = "training_step reads device values on the host: " + "; ".join(mode.reads[:3])
        acc.backward(model, loss, opt, 0)
        model.on_after_backward()
        acc.before_optimizer_step(opt)
        if t.gradient_clip_val:
            acc.clip_gradients(opt, t.gradient_clip_val)
        model.optimizer_step(t.current_epoch, batch_idx, opt, 0, None)
        model.optimizer_zero_grad(t.current_epoch, batch_idx, opt, 0)
        layout = ([(n, fx, dict(kw)) for n, _, kw, fx in calls], [k for k, _ in extra])
        vals = [loss] + [v for _, v in extra] + [v for _, v, _, _ in calls]
        if self._log_meta is None or layout == (self._log_meta, self._out_keys):
            row = torch.stack([v.detach().reshape(()).to(torch.float32) for v in vals])
            if self._ring is None:
                self._ring = torch.zeros(self.ring_rows, row.numel(), device=self.dev)
            self._ring.index_copy_(0, self._ring_pos, row.unsqueeze(0))
            self._ring_pos.add_(1).remainder_(self.ring_rows)
        return layout, vals

    def _after_step(self, replayed: bool, direct=None) -> Dict[str, torch.Tensor]:
        """Python side of one executed step: host counters, the replayed ``self.log``
        calls (ring views; ``direct``: the step's own tensors when its layout did not
        match the ring's), the step output.

        Validity window: replayed steps' outputs and logged values are VIEWS of the
        device ring (``ring_rows`` >= 2 epochs of steps), so a consumer that keeps one
        longer than two epochs sees a later step's value -- clone what must outlive
        that (the Trainer's own consumers do: ModelCheckpoint / EarlyStopping convert
        to host floats, ``defer_checkpoint`` clones its values)."""
        t = self.trainer
        if replayed:
            for gs in self.opt._rla_groups:
                gs.step += 1  # (an eager body's optimizer.step counted itself)
        if direct is not None:
            (meta, keys), vals = direct
            vals = [v.detach() for v in vals]
        else:
            meta, keys = self._log_meta, self._out_keys
            row = self._ring[self.steps_done % self.ring_rows]
            self._ring_slot_used = True
            vals = [row[j] for j in range(row.numel())]
            for v in vals:
                v._rla_fresh = True
            self.steps_done += 1
        out = {"loss": vals[0]}
        for j, k in enumerate(keys):
            out[k] = vals[1 + j]
        base = 1 + len(keys)
        for j, (name, fx, kw) in enumerate(meta):
            t._current_fx = fx
            t._log_metric(self.model, name, vals[base + j], **kw)
        t._current_fx = None
        t.callback_metrics["loss"] = vals[0]
        return out

    # ------------------------------------------------------------ capture
    def _run_eager(self, batch_fn, batch_idx: int, probe: bool):
        """One eager step (side stream on the GPU).  Returns the direct values when
        the step's logged layout does not match the ring's (then it is the last one
        on this path: ``failed``)."""
        if self._side is not None:
            self._side.wait_stream(torch.cuda.current_stream())
            try:
                with torch.cuda.stream(self._side):
                    layout, vals = self._body(batch_fn, batch_idx, probe)
            finally:
                # also on a rejection: the eager re-run reads the side stream's gather
                torch.cuda.current_stream().wait_stream(self._side)
        else:
            layout, vals = self._body(batch_fn, batch_idx, probe)
        if self._log_meta is None:
            self._log_meta, self._out_keys = layout
        elif layout != (self._log_meta, self._out_keys):
            self.reason = "the set of logged values changes between steps"
            self._give_up()
            return (layout, vals)
        if probe and self.reason is not None and self.reason.startswith("training_step reads"):
            self._give_up()
        return None

    def _capture(self, batch_fn, batch_idx: int) -> bool:
        """Record one step into a graph (nothing executes); False + ``reason`` when
        the capture fails (the step has not run: the caller runs it eagerly)."""
        groups = self.opt._rla_groups
        host_steps = [gs.step for gs in groups]
        self.arena.prepare_graph_capture()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                layout, _ = self._body(batch_fn, batch_idx)
            if layout != (self._log_meta, self._out_keys):
                raise _Unsupported("the set of logged values changes between steps")
        except Exception as e:  # noqa: BLE001 - any capture error means: stay eager
            self.reason = f"hipGraph capture failed: {e!r}"[:400]
            torch.cuda.synchronize()
            return False
        finally:
            for gs, s in zip(groups, host_steps):
                gs.step = s  # the replays count the steps
            for gs in groups:
                if gs.lr_t is not None:
                    gs.lr_host = None  # re-sync the device learning rate before the replay
            self.opt.zero_grad()  # gradients of the recorded (never executed) step
        self.graph = g
        return True

    def _step(self, batch_fn, batch_idx: int, resident: bool, static_ready: bool = False):
        """One step: capture when due, then a replay; else eager (warm-up, fallback,
        a batch the static buffers cannot hold)."""
        if self.graph is None and not self.failed and self.cuda and self.steps_done >= self.warmup \
                and (resident or static_ready):
            if not self._capture(batch_fn, batch_idx):
                self._give_up()
        if self.graph is not None and (resident or static_ready):
            for gp, gs in zip(self.opt.param_groups, self.opt._rla_groups):
                gs.sync_lr(float(gp["lr"]))
            self.graph.replay()
            self.replays += 1
            return self._after_step(replayed=True)
        direct = self._run_eager(batch_fn, batch_idx, probe=self.steps_done == 0)
        return self._after_step(replayed=False, direct=direct)

    def _give_up(self) -> None:
        if not self.failed:
            self.failed = True
            log.info(f"graph-captured training step disabled: {self.reason}")
            if self.trainer.global_rank == 0:
                print(f"[rla] graph-captured training step disabled: {self.reason}", file=sys.stderr, flush=True)

    # ----------------------------------------------------- per-batch (loader)
    def _load_static(self, batch) -> bool:
        """Copy ``batch`` into the static input buffers (the graph's inputs); False
        when its structure / shapes / dtypes differ from them."""
        leaves, spec = tree_flatten(batch)
        if self._static is None or spec != self._spec or len(leaves) != len(self._static):
            return False
        for a, b in zip(leaves, self._static):
            if not isinstance(a, torch.Tensor) or a.shape != b.shape or a.dtype != b.dtype \
                    or a.device != b.device:
                return False
        for a, b in zip(leaves, self._static):
            b.copy_(a, non_blocking=True)
        return True

    def train_batch(self, batch, batch_idx: int):
        t = self.trainer
        if isinstance(batch, tuple) and len(batch) == 2 and batch[0] == "__rla_resident__":
            if self.failed:  # rejected earlier this epoch: gather on the device, eager step
                return self._eager(self._resident_batch(), batch_idx, count_step=True)
            try:
                out = self._step(self._resident_batch, batch_idx, resident=True)
            except _Unsupported as e:
                # the batch was gathered (the cursor advanced): the eager path re-runs it
                self.reason = str(e)
                self._give_up()
                return self._eager(self._last_batch, batch_idx, count_step=True)
            t.global_step += 1
            t._update_lr_schedulers("step")
            return out
        if self.failed:
            return t._autograd_step(batch, batch_idx)
        batch = self.acc.batch_to_device(batch)
        if self._static is None and self.cuda and self.steps_done + 1 >= self.warmup:
            leaves, spec = tree_flatten(batch)
            if leaves and all(isinstance(v, torch.Tensor) and v.device == self.dev for v in leaves):
                # the inputs the capture reads; later batches are copied into them
                self._static = [torch.empty_like(v, memory_format=torch.preserve_format) for v in leaves]
                self._spec = spec
        ready = self.cuda and self.steps_done >= self.warmup and self._load_static(batch)
        if ready:
            static = tree_unflatten(self._static, self._spec)
            fn = (lambda: static)  # noqa: E731
        else:
            fn = (lambda: batch)  # noqa: E731
        try:
            out = self._step(fn, batch_idx, resident=False, static_ready=ready)
        except _Unsupported as e:
            self.reason = str(e)
            self._give_up()
            return t._autograd_step(batch, batch_idx)
        t.global_step += 1
        t._update_lr_schedulers("step")
        return out

    def _eager(self, batch, batch_idx: int, count_step: bool):
        """The Trainer's eager autograd step of an already gathered batch.
        ``count_step``: advance global_step / step schedulers (per-batch dispatch);
        a chunk's steps are counted by the Trainer after the chunk."""
        t = self.trainer
        if count_step:
            return t._autograd_step(batch, batch_idx)
        model = t.get_model()
        out = None
        for opt_idx, opt in enumerate(t.optimizers or [None]):
            out = t._optimizer_step_for(model, batch, batch_idx, opt_idx, opt, False)
        return out

    # ------------------------------------------------------- resident data
    def make_epoch_batches(self, dl, n_batches: int):
        """Resident mode: this epoch's sampler order on the device; the graph gathers
        batch ``cursor`` from the resident columns.  None: use the loader."""
        if self.failed or dl is None or dl.batch_size is None:
            return None
        from torch.utils.data._utils.collate import default_collate

        if dl.collate_fn is not default_collate:
            return None
        if self._resident is None:
            got = resident_tensors(dl.dataset, self.dev)
            if got is None:
                return None
            self._resident = got
        cols, idx_map = self._resident
        order = loader_order(dl)
        if idx_map is not None:
            order = idx_map[order]
        B = int(dl.batch_size)
        nb = min(int(n_batches), order.numel() // B)
        if nb <= 0 or (nb < n_batches and order.numel() % B):
            return None  # a partial last batch the static graph cannot gather
        order = order[: nb * B]
        assert int(order.max()) < cols[0].size(0) and int(order.min()) >= 0  # the gather trusts indices
        if self._order is None or self._order.numel() < nb * B or self._B != B:
            if self.graph is not None:
                return None  # the captured gather reads the first epoch's order buffer
            self._order = torch.empty(nb * B, dtype=torch.int64, device=self.dev)
            self._cursor = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._order[: nb * B].copy_(order.pin_memory() if self.cuda else order, non_blocking=True)
        self._cursor.zero_()
        self._B, self._nb = B, nb
        return [("__rla_resident__", i) for i in range(nb)]

    def _resident_batch(self):
        """The batch at the device cursor (gathered on the device; the cursor advances)."""
        cols, _ = self._resident
        idx = self._order.view(-1, self._B).index_select(0, self._cursor).view(self._B)
        self._cursor.add_(1)
        return [gather_rows(c, idx) for c in cols]

    @property
    def max_chunk(self) -> int:
        return max(1, self.ring_rows // 2)

    def train_chunk(self, n_steps: int):
        """``n_steps`` resident steps in one host dispatch (graph replays once captured)."""
        outs = []
        first = self.steps_done
        for _ in range(n_steps):
            if self.failed:
                outs.append(self._eager(self._resident_batch(), 0, count_step=False))
                continue
            try:
                outs.append(self._step(self._resident_batch, 0, resident=True))
            except _Unsupported as e:
                self.reason = str(e)
                self._give_up()
                outs.append(self._eager(self._last_batch, 0, count_step=False))
        k = min(n_steps, self.ring_rows)
        done = self.steps_done - first
        if self._ring is not None and done == n_steps:
            s0 = (first + n_steps - k) % self.ring_rows
            if s0 + k <= self.ring_rows:
                self._last_rows = self._ring[s0:s0 + k]
            else:
                self._last_rows = torch.cat([self._ring[s0:], self._ring[: s0 + k - self.ring_rows]])
        else:
            self._last_rows = None  # some steps logged directly: the Trainer flushes per chunk
        return outs

    def log_points(self, rows: torch.Tensor, first: int, every: int):
        """``(global step, metrics)`` of every log point among the chunk's steps."""
        base = 1 + len(self._out_keys or [])
        out = []
        for i in range(rows.size(0)):
            st = first + 1 + i
            if st % every:
                continue
            met = {}
            for j, (name, fx, kw) in enumerate(self._log_meta or []):
                training = fx.startswith("training")
                on_step = kw.get("on_step")
                on_step = training if on_step is None else on_step
                on_epoch = kw.get("on_epoch")
                on_epoch = (not training) if on_epoch is None else on_epoch
                if not on_step or not kw.get("logger", True):
                    continue
                v = rows[i, base + j]
                v._rla_fresh = True
                met[f"{name}_step" if on_epoch else name] = v
            out.append((st, met))
        return out

    # --------------------------------------------------------------- state
    def on_lr_change(self) -> None:
        pass  # read from param_groups before every replay (sync_lr)

    def eval_compatible(self, model) -> bool:
        """Validation gathers its batches on the device when the val set is resident
        (eval_epoch decides per loader; other loaders iterate as usual)."""
        return self.cuda

    def eval_epoch(self, dl, limit: int):
        """A validation pass over a RESIDENT dataset (``SyntheticImageNet``,
        ``TensorDataset``): the loader's sampler order rebuilt as a tensor (the same
        global-RNG draw as iterating it), every batch gathered on the device and run
        through ``validation_step`` / ``validation_step_end`` exactly as the loader
        path does -- no per-item CPU work, no pageable H2D copy.  Returns the step
        outputs, or None (then the Trainer iterates the loader)."""
        from torch.utils.data._utils.collate import default_collate

        if dl is None or dl.batch_size is None or dl.collate_fn is not default_collate:
            return None
        key = id(dl.dataset)
        got = self._eval_resident.get(key)
        if got is None:
            got = resident_tensors(dl.dataset, self.dev)
            if got is None:
                return None
            self._eval_resident[key] = got
        cols, idx_map = got
        order = loader_order(dl)
        if idx_map is not None:
            order = idx_map[order]
        B = int(dl.batch_size)
        n = order.numel()
        nb = n // B if dl.drop_last else -(-n // B)
        nb = min(nb, int(limit))
        if nb <= 0:
            return []
        assert int(order.max()) < cols[0].size(0) and int(order.min()) >= 0  # the gather trusts indices
        order = order[: nb * B].to(self.dev, non_blocking=False)
        t, model = self.trainer, self.model
        outs = []
        for i in range(nb):
            batch = [gather_rows(c, order[i * B:(i + 1) * B]) for c in cols]
            t._current_fx = "validation_step"
            with self.acc.autocast():
                out = model.validation_step(batch, i)
            t._current_fx = "validation_step_end"
            out = model.validation_step_end(out)
            t._current_fx = None
            if out is not None:
                outs.append(out)
        return outs

    def check(self, blocking: bool = True) -> None:
        pass

    def sync_params_to_module(self) -> None:
        self.opt.sync_host_state()  # module parameters ARE arena views

    def load_params_from_module(self) -> None:
        """After a checkpoint restore: parameters copied into the arena views, the
        optimizer's device step counter re-read (``load_state_dict``), bf16 shadow."""
        self.arena.rebind_all()
        if self.arena.bf16 is not None:
            self.arena.refresh_bf16()
        for gs in self.opt._rla_groups:
            if gs.step_t is not None:
                gs.step_t.fill_(gs.step)


class _Unsupported(RuntimeError):
    """A step the graph path cannot represent (the eager Trainer path runs it)."""


def maybe_graph_step(trainer, model) -> Optional[GraphedTrainStep]:
    if not wanted(trainer, model):
        return None
    why = static_reason(trainer, model)
    if why is not None:
        log.info(f"graph-captured training step not used: {why}")
        if trainer.global_rank == 0:
            print(f"[rla] graph-captured training step not used: {why}", file=sys.stderr, flush=True)
        trainer._graph_step_reason = why
        return None
    return GraphedTrainStep(trainer, model, warmup=int(get_config().hip_graph_warmup))
