"""``hvd.DistributedOptimizer`` with tensor fusion.

Gradient hooks (``register_post_accumulate_grad_hook``) mark parameters ready
during backward; parameters are grouped into fusion buckets (reverse order,
``HOROVOD_FUSION_THRESHOLD``, default 8 MiB -- sized for 7 xGMI links rather
than Horovod's 64 MiB NVLink default) and a full bucket is packed with ONE
multi-tensor copy launch into a fusion buffer and allreduced asynchronously
while backward continues.  Buckets launch strictly in index order so every
rank issues collectives in the same sequence (what Horovod's coordinator
negotiates).  ``synchronize()`` flushes, waits and unpacks with the 1/size
average fused into the copy.  When the parameters already live in a flat
arena, buckets are arena slices and no packing happens at all.
"""
from __future__ import annotations

import contextlib
import os
import types
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .. import ops
from ..config import get_config
from . import Average, Compression, Sum, _comm_tensor, size


class _Bucket:
    def __init__(self, params: List[torch.Tensor]):
        self.params = params
        self.pending = len(params)
        self.work = None
        self.buf: Optional[torch.Tensor] = None
        self.moved = False
        self.comm: Optional[torch.Tensor] = None
        self.table_pack = None
        self.table_unpack = None


class _FusionState:
    def __init__(self, opt, named_parameters, compression, backward_passes_per_step, op, threshold_bytes):
        self.opt = opt
        params = [p for g in opt.param_groups for p in g["params"] if p.requires_grad]
        if named_parameters is not None:
            names = {id(p): n for n, p in named_parameters}
            self.names = [names.get(id(p), f"param.{i}") for i, p in enumerate(params)]
        else:
            self.names = [f"param.{i}" for i in range(len(params))]
        self.params = params
        self.compression = compression
        self.bpps = max(1, int(backward_passes_per_step))
        self.op = op
        self.buckets: List[_Bucket] = []
        self.of: Dict[int, int] = {}
        cur, cur_b = [], 0
        for p in reversed(params):
            cur.append(p)
            cur_b += p.numel() * p.element_size()
            if cur_b >= threshold_bytes:
                self._add(cur)
                cur, cur_b = [], 0
        if cur:
            self._add(cur)
        self.next_launch = 0
        self.passes = 0
        self.skip = False
        self.synchronized = False
        # GPU ranks: the C++ fusion engine (csrc/comm/fusion_engine.cpp) packs,
        # allreduces (xGMI one-shot / RCCL) and unpacks each bucket on its own
        # thread + high-priority comm stream.  The communicator is brought up here,
        # where every rank is in lock-step; the engine itself (no collective in it)
        # only at the first bucket launch: a step that never runs autograd (the fused
        # MNIST step exchanges gradients inside its kernel) never creates its stream
        # -- an idle high-priority queue per rank made the hardware scheduler
        # time-slice two ranks sharing one GPU (Trainer.fit rehearsal, 12.8 -> 59 us
        # a step, profiles/r4_share2).
        self.engine = None
        self._engine_comm = None
        self._threshold = threshold_bytes
        if (size() > 1 and compression is Compression.none and params and params[0].is_cuda
                and get_config().hvd_native):
            from ..parallel.comm import get_native_comm

            self._engine_comm = get_native_comm()
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in params]

    def _add(self, ps):
        b = _Bucket(ps)
        for p in ps:
            self.of[id(p)] = len(self.buckets)
        self.buckets.append(b)

    def _hook(self, p: torch.Tensor) -> None:
        if size() == 1:
            return
        b = self.buckets[self.of[id(p)]]
        b.pending -= 1
        if b.pending == 0 and (self.passes + 1) % self.bpps == 0:
            self._launch_ready()

    def _launch_ready(self) -> None:
        while self.next_launch < len(self.buckets) and self.buckets[self.next_launch].pending <= 0:
            self._launch(self.buckets[self.next_launch])
            self.next_launch += 1

    def _contiguous_grads(self, b: _Bucket) -> Optional[torch.Tensor]:
        gs = [p.grad for p in b.params]
        if any(g is None or g.dtype != torch.float32 or not g.is_contiguous() for g in gs):
            return None
        srt = sorted(gs, key=lambda g: g.data_ptr())
        base = srt[0]
        end = base.data_ptr()
        for g in srt:
            if g.data_ptr() != end:
                # arena views are 4-element aligned: allow tiny padding gaps
                if not (0 <= g.data_ptr() - end < 16 and g.untyped_storage().data_ptr() ==
                        base.untyped_storage().data_ptr()):
                    return None
            end = g.data_ptr() + g.numel() * 4
        n = (end - base.data_ptr()) // 4
        storage_off = (base.data_ptr() - base.untyped_storage().data_ptr()) // 4
        flat = torch.empty(0, dtype=torch.float32, device=base.device).set_(
            base.untyped_storage(), storage_off, (n,), (1,))
        return flat

    def _launch(self, b: _Bucket) -> None:
        for p in b.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        if self.engine is None and self._engine_comm is not None:
            self.engine = self._engine_comm.fusion_engine(self._threshold)
        if self.engine is not None and all(p.grad.dtype == torch.float32 and p.grad.is_contiguous()
                                           for p in b.params):
            scale = 1.0 / size() if self.op == Average else 1.0
            b.handles = [(self.engine.submit(p.grad, scale), p.grad) for p in b.params]
            self.engine.flush()  # one fusion batch per bucket: identical on every rank
            b.work = "native"
            return
        flat = self._contiguous_grads(b) if self.compression is Compression.none else None
        if flat is not None:
            b.buf = flat
            b.table_pack = None
        else:
            n = sum(p.numel() for p in b.params)
            dt = torch.bfloat16 if self.compression is not Compression.none else torch.float32
            if b.buf is None or b.buf.numel() != n or b.buf.dtype != dt or b.table_pack is None:
                b.buf = torch.empty(n, dtype=dt, device=b.params[0].device)
                b.table_pack = "dynamic"
            pairs, off = [], 0
            for p in b.params:
                pairs.append((p.grad.reshape(-1), b.buf[off:off + p.numel()]))
                off += p.numel()
            ops.multi_copy(pairs)
        b.comm, b.moved = _comm_tensor(b.buf)
        b.work = dist.all_reduce(b.comm, op=dist.ReduceOp.SUM, async_op=True)

    def synchronize(self) -> None:
        if size() == 1:
            self.synchronized = True
            return
        for b in self.buckets:
            b.pending = 0
        self._launch_ready()
        scale = 1.0 / size() if self.op == Average else 1.0
        for b in self.buckets:
            if b.work is None:
                continue
            if b.work == "native":  # averaged in the engine's unpack
                for h, g in b.handles:
                    self.engine.wait(h, g)
                b.handles = []
                b.work = None
                continue
            b.work.wait()
            b.work = None
            if b.moved:
                b.buf.copy_(b.comm)
            if b.table_pack is None:
                if scale != 1.0:
                    ops.scale_(b.buf, scale) if b.buf.is_cuda else b.buf.mul_(scale)
            else:
                pairs, off = [], 0
                for p in b.params:
                    pairs.append((b.buf[off:off + p.numel()], p.grad.reshape(-1)))
                    off += p.numel()
                ops.multi_copy(pairs, scale=scale)
        self._reset()
        self.synchronized = True

    def _reset(self) -> None:
        for b in self.buckets:
            b.pending = len(b.params)
        self.next_launch = 0

    def on_backward_pass(self) -> None:
        self.passes += 1


def DistributedOptimizer(optimizer: torch.optim.Optimizer, named_parameters=None, compression=Compression.none,
                         backward_passes_per_step: int = 1, op=Average, gradient_predivide_factor: float = 1.0,
                         num_groups: int = 0, sparse_as_dense: bool = False):
    """Wrap ``optimizer`` IN PLACE (schedulers keep working) with fused gradient allreduce."""
    if op not in (Average, Sum):
        raise NotImplementedError(f"op {op} not supported")
    if getattr(optimizer, "_hvd_state", None) is not None:
        return optimizer
    thr = int(os.environ.get("HOROVOD_FUSION_THRESHOLD", str(8 * 1024 * 1024)))
    st = _FusionState(optimizer, list(named_parameters) if named_parameters is not None else None, compression,
                      backward_passes_per_step, op, thr)
    inner_step = optimizer.step

    def step(self, closure=None):
        if not st.skip and not st.synchronized:
            st.synchronize()
        st.synchronized = False
        self._opt_called = True
        return inner_step(closure) if closure is not None else inner_step()

    step._wrapped_by_lr_sched = True

    def synchronize(self):
        st.synchronize()

    @contextlib.contextmanager
    def skip_synchronize(self):
        st.skip = True
        try:
            yield
        finally:
            st.skip = False

    optimizer.step = types.MethodType(step, optimizer)
    optimizer.synchronize = types.MethodType(synchronize, optimizer)
    optimizer.skip_synchronize = types.MethodType(skip_synchronize, optimizer)
    optimizer._hvd_state = st
    return optimizer
