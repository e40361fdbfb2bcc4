"""``RayAccelerator``: DDP training on actor workers, one per MI355X.

Contract of the reference's ``ray_lightning/ray_ddp.py:34-295`` (SURVEY.md
§2.1 C2/C3), re-built on this framework's actor runtime and data plane:

driver (``setup``/``train``/``teardown``)
  * creates ``num_workers`` ``RayExecutor`` actors, each reserving
    ``num_cpus_per_worker`` CPUs and ONE whole GPU when ``use_gpu``; the
    runtime pins it with ``HIP_VISIBLE_DEVICES`` so every worker sees its GPU
    as device 0 (reference ray_ddp.py:94-96, :245-253);
  * forwards ``PL_GLOBAL_SEED`` (:154-159), takes the ``tcp://ip:port``
    rendezvous address from worker 0 (:161-163), maps global -> local ranks
    by node IP (:132-143), ships the trainer (:167-171), creates the 0-CPU
    queue actor inside a Tune session (:173-176), pumps results and loads
    rank 0's state dict (CPU tensors) and best checkpoint path into the
    driver's model (:184-193);
  * always tears down -- also when a worker fails (the reference leaks the
    actors on an exception).
worker (``train_remote``)
  * process group on RCCL (``nccl``) over xGMI for GPU, gloo for CPU
    (:222-237); flat-arena DDP gradient sync + fused optimizer (or the
    model's fused step); returns (results, best_path, state_dict).
"""
from __future__ import annotations

import os
import socket
import sys
from collections import defaultdict
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from .. import runtime as ray
from ..config import GPU_WORKER_REUSE_KEY, get_config
from ..lightning.accelerators import DataParallelAccelerator
from ..lightning.utilities import log
from ..session import finish_session, init_session, shutdown_session
from ..utils.timeline import mark
from ..util import Queue, process_results


@ray.remote
class RayExecutor:
    """A worker actor that runs arbitrary functions (reference ray_ddp.py:17-31)."""

    def set_env_var(self, key: str, value: str) -> None:
        os.environ[key] = value

    def set_env_vars(self, env: dict) -> None:
        vis = [k for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")
               if k in env and str(env[k]) != os.environ.get(k)]
        if vis and "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized():
            # the HIP runtime read the device list at initialisation: a late change
            # would be silently ignored and ranks would land on the wrong GPU
            raise RuntimeError(f"{vis} changed after this worker initialised HIP")
        os.environ.update({k: str(v) for k, v in env.items()})

    def get_node_ip(self) -> str:
        return ray.get_node_ip_address()

    def get_gpu_ids(self):
        return ray.get_gpu_ids()

    def execute(self, fn: Callable, *args, **kwargs):
        return fn(*args, **kwargs)

    def __rla_park__(self) -> None:
        """Reset before the runtime recycles this process for the next actor (same
        GPU): process group, native communicator, worker session and the
        process-wide config go; the HIP context, loaded kernels, imports and the
        caching allocator's memory stay (what a fresh worker would pay again)."""
        from ..config import set_config
        from ..parallel.comm import reset_native_comm

        reset_native_comm()
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
        shutdown_session()
        set_config(None)
        if "torch" in sys.modules and torch.cuda.is_initialized():
            torch.cuda.synchronize()


RECYCLE_KEY = GPU_WORKER_REUSE_KEY


def find_free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("", 0))
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        return s.getsockname()[1]


def setup_address() -> str:
    """``tcp://<node ip>:<free port>`` chosen on the calling worker's node."""
    return f"tcp://{ray.get_node_address()}:{find_free_port()}"


def _tune_session_enabled() -> bool:
    from ..tune import is_session_enabled

    return is_session_enabled()


class RayAccelerator(DataParallelAccelerator):
    """PyTorch-Lightning-style accelerator for DDP training on actor workers.

    Args:
        num_workers: number of training workers (one process per GPU).
        num_cpus_per_worker: CPUs reserved per worker (alias: ``cpus_per_worker``).
        use_gpu: reserve one whole GPU per worker and train on it (RCCL).
        init_hook: function run on every worker right after creation.
        bucket_cap_mb: DDP gradient bucket size (default 8 MiB, tuned for xGMI).
        grad_dtype: ``"fp32"`` or ``"bf16"`` gradient communication.
        config / **knobs: :class:`~ray_lightning_accelerators_amd.config.RLAConfig`
            (or individual fields, e.g. ``allreduce_algo="rccl"``); default env ``RLA_*``.
    """

    nickname = "ddp_ray"

    def __init__(self, num_workers: int = 1, num_cpus_per_worker: int = 1, use_gpu: bool = False,
                 init_hook: Optional[Callable] = None, cpus_per_worker: Optional[int] = None,
                 bucket_cap_mb: Optional[float] = None, grad_dtype: Optional[str] = None,
                 fused_optimizer: bool = True, config=None, **knobs):
        super().__init__(trainer=None, use_gpu=use_gpu, bucket_cap_mb=bucket_cap_mb, grad_dtype=grad_dtype,
                         fused_optimizer=fused_optimizer, config=config, **knobs)
        self.num_workers = int(num_workers)
        self.num_cpus_per_worker = cpus_per_worker if cpus_per_worker is not None else num_cpus_per_worker
        self.use_gpu = use_gpu
        self.init_hook = init_hook
        self.workers: List = []
        self.global_to_local: List[int] = []
        self.world_size = self.num_workers

    # ----------------------------------------------------------- driver side
    def _create_worker(self):
        opts = dict(num_cpus=self.num_cpus_per_worker, num_gpus=int(self.use_gpu))
        if self._recycles():
            # a recycled GPU worker (HIP context + kernels already loaded) when one is
            # parked for this GPU: Tune trials stop paying worker start-up each
            opts["_reuse"] = RECYCLE_KEY if self.use_gpu else RECYCLE_KEY + ":cpu"
        return RayExecutor.options(**opts).remote()

    def _recycles(self) -> bool:
        cfg = get_config()
        return cfg.reuse_workers and (self.use_gpu or cfg.reuse_cpu_workers)

    def setup(self, model) -> None:
        assert self.trainer is not None, "trainer must be attached before setup()"
        self.trainer.use_ddp = True
        self.trainer.model = model
        mark("ddp_setup")
        self.workers = [self._create_worker() for _ in range(self.num_workers)]
        if self.init_hook:
            ray.get([w.execute.remote(self.init_hook) for w in self.workers])

    def teardown(self) -> None:
        if getattr(self, "_failed", False):
            for w in self.workers:
                ray.kill(w, no_restart=True)
            self.workers = []
            self._failed = False
            return

        recycled = self._recycles()

        def shutdown_remote():
            from ..parallel.comm import reset_native_comm

            reset_native_comm()  # RCCL comm destroy + IPC unmap before the group goes
            if dist.is_available() and dist.is_initialized():
                dist.destroy_process_group()
            # a recycled worker keeps its cached blocks for the next tenant (same GPU)
            if torch.cuda.is_available() and not recycled:
                torch.cuda.empty_cache()
            shutdown_session()

        try:
            ray.get([w.execute.remote(shutdown_remote) for w in self.workers], timeout=120)
        except Exception as e:  # noqa: BLE001 - a dead worker must not block teardown
            log.warning(f"worker shutdown failed: {e!r}")
        for w in self.workers:
            ray.kill(w, no_restart=True)
        self.workers = []

    def __getstate__(self):
        d = self.__dict__.copy()
        d["workers"] = []  # actor handles never travel with the accelerator
        return d

    def __setstate__(self, d):
        d["workers"] = []
        self.__dict__.update(d)

    def get_local_ranks(self) -> List[int]:
        node_ips = ray.get([w.get_node_ip.remote() for w in self.workers])
        counter = defaultdict(int)
        out = [0] * self.num_workers
        for rank in range(self.num_workers):
            ip = node_ips[rank]
            out[rank] = counter[ip]
            counter[ip] += 1
        return out

    def train(self):
        if "PL_GLOBAL_SEED" in os.environ:
            seed = os.environ["PL_GLOBAL_SEED"]
            ray.get([w.set_env_var.remote("PL_GLOBAL_SEED", seed) for w in self.workers])
        from ..utils.faults import fault_env

        for k, v in fault_env().items():  # fault-injection tests
            ray.get([w.set_env_var.remote(k, v) for w in self.workers])
        self.ddp_address = ray.get(self.workers[0].execute.remote(setup_address))
        self.global_to_local = self.get_local_ranks()
        trainer = self.trainer
        assert trainer is not None
        mark("ddp_train_begin")
        trainer_ref = ray.put(trainer)
        mark("trainer_put")
        self.trainer = None  # do not pickle the trainer twice
        queue = None
        if _tune_session_enabled():
            queue = Queue(actor_options={"num_cpus": 0})
        try:
            futures = [self.workers[i].execute.remote(self.train_remote, trainer_ref, i, queue)
                       for i in range(self.num_workers)]
            results = process_results(futures, queue)
        except BaseException:
            # peers may be blocked inside a collective: skip the graceful shutdown
            self._failed = True
            raise
        finally:
            self.trainer = trainer
            if queue is not None:
                queue.shutdown()
        mark("ddp_results")
        results, best_path, state_dict = results[0]
        trainer.model.load_state_dict(state_dict)
        if trainer.checkpoint_callback is not None:
            trainer.checkpoint_callback.best_model_path = best_path
        return results

    # ----------------------------------------------------------- worker side
    def train_remote(self, trainer, global_rank: int, queue=None):
        mark("worker_train_remote", rank=global_rank)
        assert isinstance(self, RayAccelerator)
        self.trainer = trainer
        trainer.accelerator_backend = self
        trainer.accelerator = self
        self.global_rank = global_rank
        model = trainer.model
        if queue is not None:
            init_session(rank=global_rank, queue=queue)
        try:
            self.ddp_train(process_idx=global_rank, model=model)
        finally:
            finish_session()
        return self.results, self.best_model_path, self.model_state_dict

    def set_world_ranks(self, process_idx: int) -> None:
        self.trainer.local_rank = self.global_to_local[self.global_rank]
        self.trainer.global_rank = self.global_rank
        self.trainer.world_size = self.num_workers

    def init_ddp_connection(self, global_rank: int, world_size: int, is_slurm_managing_tasks: bool = True):
        from ..config import gpu_pg_backend

        backend = gpu_pg_backend() if self.use_gpu else "gloo"
        if not dist.is_initialized():
            log.info(f"initializing ddp: GLOBAL_RANK: {global_rank}, MEMBER: {global_rank + 1}/{world_size}")
            kw = {}
            if self.use_gpu:
                torch.cuda.set_device(0)
                if backend == "nccl" and world_size > 1:
                    # eager RCCL communicator; a world of 1 never runs a collective
                    kw["device_id"] = torch.device("cuda", 0)
            dist.init_process_group(backend=backend, init_method=self.ddp_address, rank=global_rank,
                                    world_size=world_size, **kw)

    def init_device(self, process_idx: int, is_master: bool) -> None:
        if self.use_gpu:
            # the runtime already restricted HIP_VISIBLE_DEVICES to this worker's GPU
            self.trainer.root_gpu = 0
            torch.cuda.set_device(0)
            self.root_device = torch.device("cuda", 0)
        else:
            self.root_device = torch.device("cpu")

    def get_device_ids(self):
        return [self.trainer.root_gpu] if self.use_gpu else None

    def model_to_device(self, model) -> None:
        model.to(self.root_device)
