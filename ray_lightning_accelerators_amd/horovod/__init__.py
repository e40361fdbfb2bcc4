"""Horovod-compatible collective API (``import ray_lightning_accelerators_amd.horovod as hvd``).

The subset PL's ``HorovodAccelerator`` and the reference's ``HorovodRayAccelerator``
use: ``init/rank/size/local_rank/local_size/
cross_rank/cross_size``, ``allreduce[_async][_]``, ``grouped_allreduce``,
``allgather``, ``broadcast[_]``, ``broadcast_object``, ``broadcast_parameters``,
``broadcast_optimizer_state``, ``DistributedOptimizer`` (tensor-fusion buffer,
``synchronize``/``skip_synchronize``), ``join``, ``nccl_built``.

Backend: a torch.distributed process group -- RCCL (``nccl``) over xGMI when
the worker owns a GPU, gloo otherwise -- rendezvoused through the env the
executor sets (``HOROVOD_RANK``, ``HOROVOD_SIZE``, ``HOROVOD_LOCAL_RANK``,
``HOROVOD_CROSS_RANK``, ``HOROVOD_GLOO_RENDEZVOUS_ADDR/PORT``).  The fusion
engine packs ready gradients into a flat buffer with the multi-tensor copy
kernel (one launch), allreduces it, and unpacks with the 1/size scale fused.
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import ops

Average = "Average"
Sum = "Sum"
Adasum = "Adasum"
Min = "Min"
Max = "Max"


class Compression:
    class none:  # noqa: N801
        @staticmethod
        def compress(t):
            return t, None

        @staticmethod
        def decompress(t, ctx):
            return t

    class fp16:  # noqa: N801 - bf16 on MI355X (same range as fp32, no scaling)
        @staticmethod
        def compress(t):
            return (t.to(torch.bfloat16), t.dtype) if t.is_floating_point() else (t, None)

        @staticmethod
        def decompress(t, ctx):
            return t.to(ctx) if ctx is not None else t

    bf16 = fp16


_state: Dict[str, Any] = {"initialized": False}


def _env_int(*names: str, default: int = 0) -> int:
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def init(comm=None, process_sets=None) -> None:
    if _state["initialized"]:
        return
    rank = _env_int("HOROVOD_RANK", "RANK", default=0)
    size = _env_int("HOROVOD_SIZE", "WORLD_SIZE", default=1)
    local_rank = _env_int("HOROVOD_LOCAL_RANK", "LOCAL_RANK", default=0)
    local_size = _env_int("HOROVOD_LOCAL_SIZE", "LOCAL_WORLD_SIZE", default=1)
    cross_rank = _env_int("HOROVOD_CROSS_RANK", default=0)
    cross_size = _env_int("HOROVOD_CROSS_SIZE", default=1)
    use_gpu = os.environ.get("HOROVOD_GPU_OPERATIONS", "").upper() in ("NCCL", "RCCL") or \
        (os.environ.get("RLA_HVD_USE_GPU") == "1")
    if size > 1 and not dist.is_initialized():
        addr = os.environ.get("HOROVOD_GLOO_RENDEZVOUS_ADDR", os.environ.get("MASTER_ADDR", "127.0.0.1"))
        port = os.environ.get("HOROVOD_GLOO_RENDEZVOUS_PORT", os.environ.get("MASTER_PORT", "29500"))
        from ..config import gpu_pg_backend

        kw = {}
        backend = gpu_pg_backend() if use_gpu else "gloo"
        if use_gpu:
            torch.cuda.set_device(local_rank if torch.cuda.device_count() > local_rank else 0)
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend, init_method=f"tcp://{addr}:{port}", rank=rank, world_size=size, **kw)
    _state.update(initialized=True, rank=rank, size=size, local_rank=local_rank, local_size=local_size,
                  cross_rank=cross_rank, cross_size=cross_size, use_gpu=use_gpu)


def shutdown() -> None:
    from ..parallel.comm import reset_native_comm

    reset_native_comm()
    if dist.is_initialized():
        dist.destroy_process_group()
    _state.clear()
    _state["initialized"] = False


def is_initialized() -> bool:
    return bool(_state.get("initialized"))


def _need():
    if not _state.get("initialized"):
        raise ValueError("Horovod has not been initialized; use hvd.init().")


def rank() -> int:
    _need()
    return _state["rank"]


def size() -> int:
    _need()
    return _state["size"]


def local_rank() -> int:
    _need()
    return _state["local_rank"]


def local_size() -> int:
    _need()
    return _state["local_size"]


def cross_rank() -> int:
    _need()
    return _state["cross_rank"]


def cross_size() -> int:
    _need()
    return _state["cross_size"]


def nccl_built() -> bool:
    return dist.is_nccl_available()  # RCCL on ROCm


def rocm_built() -> bool:
    return torch.version.hip is not None


def gloo_built() -> bool:
    return dist.is_gloo_available()


def mpi_built() -> bool:
    return False


def cuda_built() -> bool:
    return False


def _comm_tensor(t: torch.Tensor) -> Tuple[torch.Tensor, bool]:
    """Gloo cannot take GPU tensors; RCCL cannot take CPU tensors."""
    backend = dist.get_backend() if dist.is_initialized() else "gloo"
    if backend == "gloo" and t.is_cuda:
        return t.detach().cpu(), True
    if backend == "nccl" and not t.is_cuda:
        return t.detach().cuda(), True
    return t, False


def _op_of(average: Optional[bool], op: Optional[str]) -> str:
    if op is None:
        op = Average if (average is None or average) else Sum
    if op == Adasum:
        raise NotImplementedError("Adasum is not supported; use Average or Sum")
    return op


def _reduce_(t: torch.Tensor, op: str, prescale: float = 1.0, postscale: float = 1.0) -> torch.Tensor:
    if prescale != 1.0:
        t.mul_(prescale)
    native = None
    if size() > 1 and op in (Sum, Average) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous():
        from ..parallel.comm import get_native_comm

        native = get_native_comm()  # xGMI one-/two-shot or RCCL on the C++ engine (graph-capturable)
    if native is not None:
        native.allreduce_(t)
    elif size() > 1:
        c, moved = _comm_tensor(t)
        rop = {Sum: dist.ReduceOp.SUM, Average: dist.ReduceOp.SUM, Min: dist.ReduceOp.MIN,
               Max: dist.ReduceOp.MAX}[op]
        dist.all_reduce(c, op=rop)
        if moved:
            t.copy_(c)
    if op == Average:
        t.div_(size()) if t.is_floating_point() else t.floor_divide_(size())
    if postscale != 1.0:
        t.mul_(postscale)
    return t


def allreduce_(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
               op: Optional[str] = None, prescale_factor: float = 1.0, postscale_factor: float = 1.0,
               compression=Compression.none) -> torch.Tensor:
    _need()
    return _reduce_(tensor, _op_of(average, op), prescale_factor, postscale_factor)


def allreduce(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
              compression=Compression.none, op: Optional[str] = None, prescale_factor: float = 1.0,
              postscale_factor: float = 1.0) -> torch.Tensor:
    _need()
    c, ctx = compression.compress(tensor.detach().clone())
    out = _reduce_(c, _op_of(average, op), prescale_factor, postscale_factor)
    return compression.decompress(out, ctx)


class _Handle:
    def __init__(self, work, tensor, finalize):
        self.work = work
        self.tensor = tensor
        self.finalize = finalize

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            self.finalize()
        return self.tensor


def allreduce_async_(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
                     op: Optional[str] = None) -> _Handle:
    _need()
    o = _op_of(average, op)
    if size() == 1:
        return _Handle(None, tensor, lambda: None)
    c, moved = _comm_tensor(tensor)
    rop = {Sum: dist.ReduceOp.SUM, Average: dist.ReduceOp.SUM, Min: dist.ReduceOp.MIN, Max: dist.ReduceOp.MAX}[o]
    work = dist.all_reduce(c, op=rop, async_op=True)

    def fin():
        if moved:
            tensor.copy_(c)
        if o == Average:
            tensor.div_(size())

    return _Handle(work, tensor, fin)


def allreduce_async(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
                    op: Optional[str] = None) -> _Handle:
    return allreduce_async_(tensor.detach().clone(), average, name, op)


def synchronize(handle: _Handle) -> torch.Tensor:
    return handle.wait()


def poll(handle: _Handle) -> bool:
    return handle.work is None or handle.work.is_completed()


def grouped_allreduce(tensors: Sequence[torch.Tensor], average: Optional[bool] = None,
                      op: Optional[str] = None) -> List[torch.Tensor]:
    outs = [t.detach().clone() for t in tensors]
    _fused_allreduce_(outs, _op_of(average, op))
    return outs


def grouped_allreduce_(tensors: Sequence[torch.Tensor], average: Optional[bool] = None,
                       op: Optional[str] = None) -> List[torch.Tensor]:
    _fused_allreduce_(list(tensors), _op_of(average, op))
    return list(tensors)


def _fused_allreduce_(tensors: List[torch.Tensor], op: str) -> None:
    """Tensor fusion: pack -> ONE collective -> unpack (+1/size) with the copy kernel."""
    _need()
    if not tensors:
        return
    if size() == 1 and op != Average:
        return
    floats = [t for t in tensors if t.dtype == torch.float32 and t.is_contiguous()]
    others = [t for t in tensors if not (t.dtype == torch.float32 and t.is_contiguous())]
    if floats:
        n = sum(t.numel() for t in floats)
        buf = torch.empty(n, dtype=torch.float32, device=floats[0].device)
        pairs, off = [], 0
        for t in floats:
            pairs.append((t.reshape(-1), buf[off:off + t.numel()]))
            off += t.numel()
        ops.multi_copy(pairs)
        if size() > 1:
            c, moved = _comm_tensor(buf)
            dist.all_reduce(c, op=dist.ReduceOp.SUM if op in (Sum, Average) else
                            (dist.ReduceOp.MIN if op == Min else dist.ReduceOp.MAX))
            if moved:
                buf.copy_(c)
        scale = 1.0 / size() if op == Average else 1.0
        ops.multi_copy([(b, t) for t, b in pairs], scale=scale)
    for t in others:
        _reduce_(t, op)


def allgather(tensor: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    """Concatenate every rank's tensor along dim 0 (first dims may differ)."""
    _need()
    if size() == 1:
        return tensor.detach().clone()
    c, moved = _comm_tensor(tensor.detach().contiguous())
    n = torch.tensor([c.shape[0] if c.dim() else 1], device=c.device, dtype=torch.int64)
    ns = [torch.zeros_like(n) for _ in range(size())]
    dist.all_gather(ns, n)
    sizes = [int(x.item()) for x in ns]
    mx = max(sizes)
    pad_shape = (mx,) + tuple(c.shape[1:]) if c.dim() else (mx,)
    padded = torch.zeros(pad_shape, dtype=c.dtype, device=c.device)
    padded[: sizes[rank()]] = c if c.dim() else c.reshape(1)
    outs = [torch.empty_like(padded) for _ in range(size())]
    dist.all_gather(outs, padded)
    res = torch.cat([o[:s] for o, s in zip(outs, sizes)], dim=0)
    return res.to(tensor.device) if moved else res


def allgather_object(obj: Any, name: Optional[str] = None) -> List[Any]:
    _need()
    if size() == 1:
        return [obj]
    out = [None] * size()
    dist.all_gather_object(out, obj)
    return out


def broadcast_(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> torch.Tensor:
    _need()
    if size() > 1:
        c, moved = _comm_tensor(tensor)
        dist.broadcast(c, root_rank)
        if moved:
            tensor.copy_(c)
    return tensor


def broadcast(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> torch.Tensor:
    return broadcast_(tensor.detach().clone(), root_rank, name)


def broadcast_object(obj: Any, root_rank: int = 0, name: Optional[str] = None) -> Any:
    _need()
    if size() == 1:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=root_rank)
    return box[0]


def broadcast_parameters(params, root_rank: int = 0) -> None:
    """Broadcast a state_dict / named_parameters / list of (name, tensor) from root."""
    if isinstance(params, dict):
        items = sorted(params.items())
    elif isinstance(params, Iterable):
        items = list(params)
    else:
        raise ValueError("invalid params of type %s" % type(params))
    tensors = [p for _, p in items if isinstance(p, torch.Tensor)]
    for t in tensors:
        broadcast_(t.data if hasattr(t, "data") else t, root_rank)


def broadcast_optimizer_state(optimizer: torch.optim.Optimizer, root_rank: int = 0) -> None:
    state = broadcast_object(optimizer.state_dict() if rank() == root_rank else None, root_rank)
    if rank() != root_rank:
        optimizer.load_state_dict(state)
    # keep hyper-parameters identical too (e.g. the LR scaled by hvd.size())
    for g_local, g_root in zip(optimizer.param_groups, state["param_groups"]):
        for k, v in g_root.items():
            if k != "params":
                g_local[k] = v


def join(device: int = -1) -> int:
    """Barrier; returns the rank that joined last (here: size-1, deterministic)."""
    _need()
    if size() > 1:
        dist.barrier()
    return size() - 1


def barrier() -> None:
    _need()
    if size() > 1:
        dist.barrier()


from .optimizer import DistributedOptimizer  # noqa: E402,F401
