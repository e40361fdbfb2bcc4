"""Accelerator base classes (the PL 1.1 accelerator contract the reference
subclasses: ``DDPSpawnAccelerator`` for RayAccelerator, ``HorovodAccelerator``
for HorovodRayAccelerator).

The driver-side protocol is ``setup(model) -> train() -> teardown()``; the
worker-side helpers (device placement, optimizer fusion, DDP gradient sync,
collectives for metrics / early stopping) are shared by all accelerators.
"""
from __future__ import annotations

import contextlib
import os
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from ..config import RLAConfig, get_config, log_config, set_config
from ..utils.timeline import mark
from .utilities import log, move_to_device, rank_zero_only_state, seed_everything


def _dist_active() -> bool:
    """A process group with more than one rank (a world of 1 needs no collective --
    and an RCCL group of 1 would create its communicator, ~1 s, on the first one)."""
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class Accelerator:
    """Single-process accelerator (CPU, or one GPU)."""

    nickname = "single"

    def __init__(self, trainer=None, use_gpu: Optional[bool] = None, fused_optimizer: bool = True):
        self.trainer = trainer
        self.use_gpu = use_gpu
        self.fused_optimizer = fused_optimizer
        self.root_device = torch.device("cpu")
        self.arena = None
        self.sync = None
        self.ddp_plugin = None

    # ------------------------------------------------------------ driver side
    def setup(self, model) -> None:
        t = self.trainer
        t.accelerator_backend = self
        if self.use_gpu is None:
            self.use_gpu = t.gpus > 0
        t.model = model

    def train(self):
        t = self.trainer
        model = t.model
        self.init_device(0, True)
        self.model_to_device(model)
        return t._run(model)

    def teardown(self) -> None:
        pass

    # ------------------------------------------------------------ device
    def init_device(self, process_idx: int, is_master: bool) -> None:
        if self.use_gpu:
            if not torch.cuda.is_available():
                raise RuntimeError("use_gpu=True but no GPU is visible to this process")
            idx = self.trainer.root_gpu if self.trainer.root_gpu is not None else 0
            torch.cuda.set_device(idx)
            self.trainer.root_gpu = idx
            self.root_device = torch.device("cuda", idx)
        else:
            self.root_device = torch.device("cpu")

    def model_to_device(self, model) -> None:
        model.to(self.root_device)

    def get_device_ids(self) -> Optional[List[int]]:
        return [self.trainer.root_gpu] if self.use_gpu else None

    def batch_to_device(self, batch: Any) -> Any:
        dm = self.trainer.datamodule
        if dm is not None and type(dm).transfer_batch_to_device is not type(dm).__mro__[-2].__dict__.get(
                "transfer_batch_to_device", None) and hasattr(dm, "transfer_batch_to_device"):
            return dm.transfer_batch_to_device(batch, self.root_device)
        return move_to_device(batch, self.root_device)

    @contextlib.contextmanager
    def autocast(self):
        prec = self.trainer.precision
        if prec in ("bf16", 16, "16") and self.root_device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                yield
        elif prec == "bf16":
            with torch.autocast("cpu", dtype=torch.bfloat16):
                yield
        else:
            yield

    # ------------------------------------------------------------ optimizers
    def setup_optimizers(self, model, optimizers, schedulers):
        from ..parallel.arena import ParamArena
        from ..parallel.fused_optim import can_fuse, fuse_optimizer

        params = [p for p in model.parameters() if p.requires_grad]
        fusable = bool(params) and all(p.dtype == torch.float32 for p in params) and \
            len({p.device for p in params}) == 1
        if fusable:
            try:
                self.arena = ParamArena(model, params)
            except ValueError:
                self.arena = None
        if self.arena is not None and self.fused_optimizer and get_config().fused_optimizer:
            fused = False
            for opt in optimizers:
                if can_fuse(opt, self.arena):
                    fuse_optimizer(opt, self.arena, grad_scale_fn=lambda: self.grad_scale)
                    fused = True
            from ..ops.shadow import wants_shadow

            if fused and self.arena.device.type == "cuda" and wants_shadow(model):
                self.arena.enable_bf16_shadow(model)  # the fused step writes bf16 weights too
        return optimizers, schedulers

    @property
    def grad_scale(self) -> float:
        return self.sync.grad_scale if self.sync is not None else 1.0

    def configure_ddp(self, model) -> None:
        """Single process: nothing to synchronise."""
        self.sync = None

    def before_forward(self, sync: bool = True) -> None:
        if self.sync is not None:
            self.sync.prepare_for_backward(sync)

    def backward(self, model, loss, optimizer, optimizer_idx: int = 0) -> None:
        model.backward(loss, optimizer, optimizer_idx)

    def before_optimizer_step(self, optimizer) -> None:
        if self.sync is not None:
            self.sync.finish()

    def clip_gradients(self, optimizer, max_norm: float) -> None:
        if self.arena is not None:
            from .. import ops

            self.arena.gather_grads()  # stolen (non-arena) grads first
            norm = ops.sumsq(self.arena.grad).sqrt() * self.grad_scale
            coef = (max_norm / (norm + 1e-6)).clamp(max=1.0)
            self.arena.grad.mul_(coef)
        else:
            params = [p for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
            torch.nn.utils.clip_grad_norm_(params, max_norm)

    # ------------------------------------------------------------ collectives
    @property
    def require_distributed_sampler(self) -> bool:
        return False

    @property
    def distributed_sampler_kwargs(self) -> dict:
        return {}

    def barrier(self, name: Optional[str] = None) -> None:
        if _dist_active():
            dist.barrier()

    def broadcast(self, obj: Any, src: int = 0) -> Any:
        if not _dist_active():
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src)
        return box[0]

    def sync_tensor(self, tensor: torch.Tensor, group=None, reduce_op: Any = "mean") -> torch.Tensor:
        if not _dist_active():
            return tensor
        t = tensor.clone().to(self._comm_device())
        op = str(reduce_op).lower()
        if op in ("max",):
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elif op in ("min",):
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            if op in ("mean", "avg"):
                t = t / dist.get_world_size()
        return t.to(tensor.device)

    def all_gather(self, tensor: torch.Tensor) -> torch.Tensor:
        if not _dist_active():
            return tensor.unsqueeze(0)
        t = tensor.to(self._comm_device())
        out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        return torch.stack(out).to(tensor.device)

    def early_stopping_should_stop(self, should_stop: bool) -> bool:
        if not _dist_active():
            return should_stop
        t = torch.tensor([1.0 if should_stop else 0.0], device=self._comm_device())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return bool(t.item() >= 1.0)  # PL: stop when any rank wants to stop

    def _comm_device(self) -> torch.device:
        if dist.is_initialized() and dist.get_backend() == "nccl":
            return self.root_device
        return torch.device("cpu")


_fits_in_process = 0


def _ckpt_takeovers() -> int:
    from . import utilities

    return int(getattr(utilities, "writer_takeovers", 0))


def _worker_diag(trainer) -> None:
    """``RLA_WORKER_DIAG_DIR``: one JSON line per fit and rank (worker reuse audit,
    scripts/bench_tune.py --diag): process id, how many fits this process has run
    (> 1: a recycled worker), the native communicator this fit used (a fresh one per
    fit: its Python id and bring-up state) and how often the fused step's exchange
    region was re-armed in it."""
    global _fits_in_process
    _fits_in_process += 1
    d = os.environ.get("RLA_WORKER_DIAG_DIR")
    if not d:
        return
    import json

    from ..parallel.comm import get_native_comm

    comm = get_native_comm(create=False)
    eng = getattr(getattr(trainer, "_fused", None), "eng", None)
    rec = {"pid": os.getpid(), "fit_in_process": _fits_in_process, "rank": trainer.global_rank,
           "world": trainer.world_size, "cwd": os.getcwd(),
           "comm_id": comm.serial if comm is not None else None,
           "comm": comm.describe() if comm is not None else None,
           "comm_error_state": int(comm._c.error_state()) if comm is not None else None,
           "dp_region_rearms": getattr(comm, "rearms", 0) if comm is not None else 0,
           "fused_dp": bool(eng is not None and eng.dp_ctx is not None and eng.one_launch_dp),
           "dp_proto": getattr(eng, "dp_proto", None) if eng is not None else None,
           "global_step": trainer.global_step,
           "ckpt_writer_takeovers": _ckpt_takeovers()}
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"fit_{os.getpid()}_{_fits_in_process}_r{trainer.global_rank}.json"), "w") as f:
        json.dump(rec, f)


class DataParallelAccelerator(Accelerator):
    """Shared worker-side flow of process-per-device data parallelism.

    ``ddp_train`` mirrors PL 1.1 ``DDPSpawnAccelerator.ddp_train`` (SURVEY.md
    §2.2 U2): seed, world ranks, process group, setup hook, device, model to
    device, optimizers, DDP wrapping, train_or_test, hand-back of state.
    """

    nickname = "ddp"

    def __init__(self, trainer=None, use_gpu: bool = False, bucket_cap_mb: Optional[float] = None,
                 grad_dtype: Optional[str] = None, fused_optimizer: bool = True,
                 config: Optional[RLAConfig] = None, **knobs):
        """``bucket_cap_mb`` / ``grad_dtype`` / any other :class:`RLAConfig` field
        (``allreduce_algo=...``, ``use_hip_graph=...``) override ``config`` (default:
        env ``RLA_*``); the resolved config travels to the workers."""
        super().__init__(trainer, use_gpu=use_gpu, fused_optimizer=fused_optimizer)
        self.global_rank = 0
        self.world_size = 1
        base = config if config is not None else RLAConfig.from_env()
        self.config = base.replace(**{k: v for k, v in dict(bucket_cap_mb=bucket_cap_mb, grad_dtype=grad_dtype,
                                                             **knobs).items() if v is not None})
        self.bucket_cap_mb = self.config.bucket_cap_mb
        self.grad_dtype = self.config.grad_dtype
        self.ddp_address: Optional[str] = None
        self.results = None
        self.model_state_dict = None
        self.best_model_path = None

    # hooks for subclasses
    def set_world_ranks(self, process_idx: int) -> None:
        self.trainer.global_rank = self.global_rank
        self.trainer.world_size = self.world_size

    def init_ddp_connection(self, global_rank: int, world_size: int) -> None:
        raise NotImplementedError

    @property
    def require_distributed_sampler(self) -> bool:
        return True

    @property
    def distributed_sampler_kwargs(self) -> dict:
        kw = dict(num_replicas=self.world_size, rank=self.global_rank)
        if self.ddp_plugin is not None and hasattr(self.ddp_plugin, "distributed_sampler_kwargs"):
            kw = self.ddp_plugin.distributed_sampler_kwargs(kw)
        return kw

    def configure_ddp(self, model) -> None:
        from ..parallel.ddp import GradSynchronizer, default_bucket_cap_mb

        if self.arena is None or self.world_size <= 1 or not dist.is_initialized():
            self.sync = None
            return
        fused = any(getattr(o, "_rla_fused", False) for o in self.trainer.optimizers)
        if self.arena.data.is_cuda and get_config().native_comm:
            # bring the native data plane (RCCL + validated xGMI one-shot) up on every
            # rank together, before backward hooks start issuing collectives
            from ..parallel.comm import get_native_comm

            get_native_comm()
        self.sync = GradSynchronizer(
            model, self.arena, bucket_cap_mb=self.bucket_cap_mb or default_bucket_cap_mb(),
            grad_dtype=self.grad_dtype, average_in_optimizer=fused)
        self.sync.broadcast_parameters(0)

    def ddp_train(self, process_idx: int, model):
        from ..utils.faults import hang_watch_start, hang_watch_stop

        watch = hang_watch_start(f"fit{_fits_in_process + 1}")
        try:
            return self._ddp_train(process_idx, model)
        finally:
            hang_watch_stop(watch)

    def _ddp_train(self, process_idx: int, model):
        t = self.trainer
        set_config(self.config)  # every rank runs the driver-resolved knobs
        if "PL_GLOBAL_SEED" in os.environ:
            seed_everything(int(os.environ["PL_GLOBAL_SEED"]))
        self.set_world_ranks(process_idx)
        rank_zero_only_state.rank = t.global_rank
        if t.global_rank == 0 and get_config().async_checkpoint:
            # the checkpoint writer process, forked now -- before this process
            # touches a GPU, so it starts in milliseconds (torch already imported)
            from .utilities import process_checkpoint_writer

            process_checkpoint_writer()
        mark("pg_init_begin", rank=t.global_rank)
        self.init_ddp_connection(t.global_rank, t.world_size)
        mark("pg_init_end", rank=t.global_rank)
        log_config(t.global_rank, self.config)
        self.init_device(process_idx, t.global_rank == 0)
        mark("device_ready", rank=t.global_rank)
        if t.sync_batchnorm and t.world_size > 1 and dist.is_initialized():
            # PL: Trainer(sync_batchnorm=True) -> BN statistics all-reduced across ranks
            # (fused BN+ReLU layers stay fused and all-reduce their per-channel sums)
            from ..ops.bn import convert_sync_batchnorm

            convert_sync_batchnorm(model)
        self.model_to_device(model)
        mark("model_on_device", rank=t.global_rank)
        results = t._run(model)
        mark("run_end", rank=t.global_rank)
        _worker_diag(t)
        self.transfer_distrib_spawn_state_on_fit_end(model, results)
        mark("state_handed_back", rank=t.global_rank)
        return results

    def transfer_distrib_spawn_state_on_fit_end(self, model, results) -> None:
        t = self.trainer
        self.results = results
        # CPU tensors (the reference ships device tensors back, ray_ddp.py:274)
        self.model_state_dict = t._model_state_dict(model)
        cb = t.checkpoint_callback
        self.best_model_path = cb.best_model_path if cb is not None else None


class DDPAccelerator(DataParallelAccelerator):
    """Process group from the environment (``torchrun``-launched scripts)."""

    nickname = "ddp_env"

    def setup(self, model) -> None:
        t = self.trainer
        t.accelerator_backend = self
        t.use_ddp = True
        t.model = model
        self.world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self.global_rank = int(os.environ.get("RANK", "0"))
        if self.use_gpu is None:
            self.use_gpu = t.gpus > 0

    def set_world_ranks(self, process_idx: int) -> None:
        super().set_world_ranks(process_idx)
        self.trainer.local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    def init_device(self, process_idx: int, is_master: bool) -> None:
        if self.use_gpu:
            self.trainer.root_gpu = self.trainer.local_rank
        super().init_device(process_idx, is_master)

    def init_ddp_connection(self, global_rank: int, world_size: int) -> None:
        if world_size > 1 and not dist.is_initialized():
            from ..config import gpu_pg_backend

            backend = gpu_pg_backend() if self.use_gpu else "gloo"
            kw = {}
            if self.use_gpu and backend == "nccl":
                kw["device_id"] = torch.device("cuda", self.trainer.local_rank)
            dist.init_process_group(backend, rank=global_rank, world_size=world_size, **kw)

    def train(self):
        return self.ddp_train(self.global_rank, self.trainer.model)


def resolve_accelerator(trainer) -> Accelerator:
    acc = trainer.accelerator
    if isinstance(acc, Accelerator):
        return acc
    if hasattr(acc, "setup") and hasattr(acc, "train") and not isinstance(acc, str):
        return acc  # duck-typed accelerator
    name = (acc or trainer.distributed_backend or "").lower() if isinstance(acc, (str, type(None))) else ""
    use_gpu = trainer.gpus > 0
    if name in ("ddp", "ddp_env") or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return DDPAccelerator(trainer, use_gpu=use_gpu)
    if name in ("ddp_ray", "ray"):
        from ..accelerators.ray_ddp import RayAccelerator

        return RayAccelerator(num_workers=max(1, trainer.gpus or 1), use_gpu=use_gpu)
    if name in ("horovod_ray",):
        from ..accelerators.ray_horovod import HorovodRayAccelerator

        return HorovodRayAccelerator(num_slots=max(1, trainer.gpus or 1), use_gpu=use_gpu)
    return Accelerator(trainer, use_gpu=use_gpu)
