"""Fused BatchNorm (+ReLU) (+residual add) for NHWC bf16 activations.

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` (same parameters, buffers
and state-dict keys, so Lightning checkpoints are interchangeable) whose
forward is ``act(bn(x) + residual)``.  On an MI355X with channels_last bf16
activations (ResNet-50 under bf16 autocast) it runs the gfx950 kernels of
``csrc/bn_act.hip``:

  forward   partial sums (1 read of x) -> finalize ([C]; running stats and
            num_batches_tracked updated in-kernel) -> apply (read x [+res], write y)
  backward  partial sums (read x, dy [, y]) -> finalize -> apply (write dx)
            (without a residual the ReLU mask is recomputed from x and the
            forward's scale/shift, so y is not re-read; with one, the partial
            pass writes dres = the masked gradient and the apply reads x, dres)

which replaces MIOpen's six batch-norm kernels per layer plus the separate
ReLU, residual-add and ReLU-backward passes (profiles/r1_resnet50_v2).

Residual-gradient fold: when the residual of one fused layer is the OUTPUT of
another fused layer (ResNet's identity shortcut: block k adds block k-1's
output), autograd would sum the two gradients of that tensor (the next conv's
dgrad and this layer's dres) in a separate add kernel (read 2, write 1 over the
activation).  Instead the residual enters the autograd graph detached, this
layer's backward parks dres in the producer's ``_FoldSlot``, and the producer's
backward kernels read it as a second incoming gradient (``dy2``).  The chain
conv1 -> bn1 -> ... -> bn3 of the consumer guarantees its backward runs first.

``Trainer(sync_batchnorm=True)`` goes through :func:`convert_sync_batchnorm`,
which keeps the fusion and all-reduces the per-channel sums (SyncBatchNorm
semantics: global statistics, local weight/bias gradients).

Anything the kernels do not cover (CPU, fp32 / NCHW input, C % 8 != 0 or
C > 2048, eval with autograd) runs the plain PyTorch composition.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from . import require, use_native

MAX_C = 2048
stats = {"fused": 0, "fallback": 0}


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1)


def fused_ok(x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.numel() > 0):
        return False
    c = x.size(1)
    if c % 8 or c > MAX_C or not _nhwc(x).is_contiguous() or x.data_ptr() % 16:
        return False
    if residual is not None:
        if residual.shape != x.shape or residual.dtype != torch.bfloat16 or not _nhwc(residual).is_contiguous() \
                or residual.data_ptr() % 16:
            return False
    return use_native(x)


class _FoldSlot:
    """Hand-off of a consumer layer's residual gradient to the producer of that residual."""

    __slots__ = ("dres", "claimed", "x3", "bwd_part", "bwd_d")

    def __init__(self):
        self.dres = None
        self.claimed = False
        self.x3 = None        # this layer's input, for a consumer conv fusing our backward partial
        self.bwd_part = None  # that conv's partial sums of d (ops.conv fuse_bn_dgrad)
        self.bwd_d = None     # the d those sums are of (the tensor the conv returned as our dy)


fold_stats = {"folded": 0, "fused_rejected": 0, "deferred": 0, "materialized": 0}


def defer_enabled() -> bool:
    """``RLA_BN_DEFER=0`` keeps every BatchNorm's apply pass (see :class:`DeferredApply`)."""
    return os.environ.get("RLA_BN_DEFER", "1") != "0"


class DeferredApply:
    """A BatchNorm + ReLU whose apply pass was left to its consumer (ResNet's bn2, read
    only by conv3): the layer returns its INPUT x (an autograd alias standing for
    relu(x * scale + shift)) tagged ``_rla_pre`` with this record, and a 1x1 conv that
    understands it applies the map to its operand fragments (csrc/conv1x1.hip PRE,
    csrc/conv_wgrad.hip PRE) -- the [M, C] activation is never written or re-read.
    Any other consumer must call :func:`materialize` first.  ``nbt``: the
    num_batches_tracked increment the skipped apply kernel would have made (when the
    statistics came from a conv epilogue), taken by whichever kernel applies the map."""

    __slots__ = ("st", "nbt", "used")

    def __init__(self):
        self.st = None
        self.nbt = None
        self.used = False

    def take_nbt(self):
        n, self.nbt = self.nbt, None
        return n


class _MaterializeFn(torch.autograd.Function):
    """relu(x * scale + shift) of a deferred BatchNorm output, for a consumer that cannot
    apply it itself; the gradient passes through unchanged (the deferred tensor already
    stands for the activation in the autograd graph)."""

    @staticmethod
    def forward(ctx, x, pre):
        y = torch.empty_like(x, memory_format=torch.channels_last)
        require().bn_apply(_nhwc(x), pre.st[2], pre.st[3], None, True, _nhwc(y), pre.take_nbt())
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, None


def materialize(x: torch.Tensor) -> torch.Tensor:
    """The real activation of a possibly deferred BatchNorm output (no-op otherwise)."""
    pre = getattr(x, "_rla_pre", None)
    if pre is None:
        return x
    fold_stats["materialized"] += 1
    return _MaterializeFn.apply(x, pre)


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu, group,
                slot=None, sink=None, part=None, pool=None, defer=None):
        # slot: this layer's own _FoldSlot (a consumer may park dres for our backward);
        # sink: the producer slot of `residual` (residual is then passed detached);
        # part: partial sums the producing conv computed in its epilogue (ops.conv.BNStats);
        # pool: (k, s, pad) of a max pool applied to relu(bn(x)) in the same pass (the
        # ResNet stem): the normalised activation is never written, the output is pooled
        mod = require()
        C = x.size(1)
        xv = _nhwc(x)
        count = float(xv.numel() // C)
        # num_batches_tracked: += 1 by the partial kernel, or -- with the conv's partials
        # -- by the apply kernel, after a finalize told to use the incremented value
        pending = part is not None and nbt is not None
        if part is None:
            part = mod.bn_partial(xv, None, None, C, 0, False, nbt)
        if group is not None:
            # SyncBatchNorm: global per-channel sums (equal per-rank batches, as the
            # DistributedSampler shards are)
            part = part.sum(0, keepdim=True)
            dist.all_reduce(part, group=group)
            count *= dist.get_world_size(group)
        st = mod.bn_finalize(part, count, weight, bias, running_mean, running_var, nbt, momentum, eps, pending)
        if pool is not None:
            # pooled bf16(relu(x * scale + shift)) + one-byte argmax (csrc/pool.hip BN); the
            # backward scatters through the argmax, then runs the usual recomputed-mask pass
            k, s_, pad = pool
            yp, arg = mod.maxpool_fwd(xv, k, s_, pad, st, nbt if pending else None)
            ctx.relu, ctx.has_res, ctx.group, ctx.count = True, False, group, count
            ctx.slot, ctx.sink, ctx.recomp = slot, sink, True
            ctx.pool = (x.size(2), x.size(3), k, s_, pad)
            ctx.save_for_backward(x, None, weight, st, arg)
            return yp.permute(0, 3, 1, 2)
        ctx.pool = None
        if defer is not None:
            # the consumer applies relu(x * scale + shift) itself (DeferredApply): x stands
            # for the activation; the backward is the usual recomputed-mask one
            defer.st, defer.nbt = st, (nbt if pending else None)
            ctx.relu, ctx.has_res, ctx.group, ctx.count = True, False, group, count
            ctx.slot, ctx.sink, ctx.recomp = slot, sink, True
            ctx.save_for_backward(x, None, weight, st, None)
            return x
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mod.bn_apply(xv, st[2], st[3], _nhwc(residual) if residual is not None else None, relu, _nhwc(y),
                     nbt if pending else None)
        ctx.relu, ctx.has_res, ctx.group, ctx.count = relu, residual is not None, group, count
        ctx.slot, ctx.sink = slot, sink
        if slot is not None and relu and residual is not None and group is None:
            slot.x3 = x  # a 1x1 conv reading y may compute our backward partial (ops/conv.py)
        # ReLU without a residual: the backward recomputes the mask x*scale+shift > 0
        # from the stats (one stream less to read in both backward passes); with a
        # residual the mask needs the sum, so y is kept
        ctx.recomp = relu and residual is None
        ctx.save_for_backward(x, y if relu and not ctx.recomp else None, weight, st, None)
        return y

    @staticmethod
    def backward(ctx, dy):
        mod = require()
        x, y, weight, st, arg = ctx.saved_tensors
        mean, invstd = st[0], st[1]
        ss = st if ctx.recomp else None
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if ctx.pool is not None:
            # dy is the POOLED output's gradient: both backward passes gather relu(bn(x))'s
            # gradient through the argmax bytes themselves (csrc/pool_gather.h) -- the
            # 205 MB maxpool_bwd output is never written or read
            geo = list(ctx.pool)
            dyp = dy.permute(0, 2, 3, 1)
            part = mod.bn_partial(_nhwc(x), None, dyp, x.size(1), 1, True, None, None, st, None, arg, geo)
            if ctx.group is not None:
                local = mod.bn_bwd_finalize(part, ctx.count, weight, mean, invstd)
                part = part.sum(0, keepdim=True)
                dist.all_reduce(part, group=ctx.group)
            else:
                local = None
            coef = mod.bn_bwd_finalize(part, ctx.count, weight, mean, invstd)
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            mod.bn_bwd_apply(_nhwc(x), None, dyp, coef, True, _nhwc(dx), None, None, st, arg, geo)
            wsrc = local if local is not None else coef
            dgamma = wsrc[0] if weight is not None and ctx.needs_input_grad[1] else None
            dbeta = wsrc[1] if ctx.needs_input_grad[2] else None
            return dx, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None, None, None
        C = x.size(1)
        xv, dyv = _nhwc(x), _nhwc(dy)
        yv = _nhwc(y) if y is not None else None
        dy2 = None
        if ctx.slot is not None and ctx.slot.dres is not None:
            dy2, ctx.slot.dres = _nhwc(ctx.slot.dres), None
            fold_stats["folded"] += 1
        # residual layer: dres is the masked incoming gradient d itself -- the partial
        # pass writes it, and the apply pass reads x and d only (csrc/bn_act.hip, WD)
        fused = ctx.slot.bwd_part if ctx.slot is not None else None
        if fused is not None:
            # the conv's partial sums are of ITS d: valid only when that tensor arrives
            # here unchanged -- another autograd consumer of our output (a hook, a
            # feature tap) makes autograd pass d + g instead, and the partial pass then
            # runs over the sum (dres is already inside d, so no dy2: ADVICE r4)
            d_ref, ctx.slot.bwd_d = ctx.slot.bwd_d, None
            if d_ref is None or d_ref.data_ptr() != dy.data_ptr() or d_ref.shape != dy.shape:
                ctx.slot.bwd_part, fused = None, None
                fold_stats["fused_rejected"] += 1
        if fused is not None:
            # the consumer 1x1 conv's input-gradient kernel already produced d (= dy here)
            # and its partial sums (ops/conv.py fuse_bn_dgrad)
            ctx.slot.bwd_part, part, dres = None, fused, dy
        else:
            dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res else None
            part = mod.bn_partial(xv, yv, dyv, C, 1, ctx.relu, None, dy2, ss,
                                  _nhwc(dres) if dres is not None else None)
        local = None
        if ctx.group is not None:
            local = mod.bn_bwd_finalize(part, ctx.count, weight, mean, invstd)  # local dgamma / dbeta
            part = part.sum(0, keepdim=True)
            dist.all_reduce(part, group=ctx.group)
        coef = mod.bn_bwd_finalize(part, ctx.count, weight, mean, invstd)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        if dres is not None:
            mod.bn_bwd_apply(xv, None, _nhwc(dres), coef, False, _nhwc(dx), None)
        else:
            mod.bn_bwd_apply(xv, yv, dyv, coef, ctx.relu, _nhwc(dx), None, dy2, ss)
        if ctx.sink is not None:
            ctx.sink.dres, dres = dres, None  # the producer's backward consumes it
        wsrc = local if local is not None else coef
        # views of the coefficient tensor (no copy kernels): autograd hands them to .grad
        dgamma = wsrc[0] if weight is not None and ctx.needs_input_grad[1] else None
        dbeta = wsrc[1] if ctx.needs_input_grad[2] else None
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, None, None


class BatchNormAct2d(nn.BatchNorm2d):
    """``act(BatchNorm2d(x) + residual)`` with ``act`` in {"relu", None}."""

    def __init__(self, num_features: int, act: Optional[str] = "relu", eps: float = 1e-5,
                 momentum: Optional[float] = 0.1, affine: bool = True, track_running_stats: bool = True,
                 device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device=device, dtype=dtype)
        if act not in ("relu", None):
            raise ValueError(f"act must be 'relu' or None, got {act!r}")
        self.act = act
        self.sync = False
        self.process_group = None
        self._warned = False
        self.fold_residual_grad = True  # see the module docstring

    def _pool_geometry(self, pool, residual):
        k, s, p = getattr(pool, "kernel_size", None), getattr(pool, "stride", None), getattr(pool, "padding", None)
        if (self.act == "relu" and residual is None and isinstance(pool, nn.MaxPool2d) and isinstance(k, int)
                and isinstance(s, int) and isinstance(p, int) and pool.dilation == 1 and not pool.ceil_mode
                and not pool.return_indices and 2 * p <= k and 1 <= k <= 15 and s >= 1):
            return (k, s, p)
        return None

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={self.act}, sync={self.sync}"

    def _group(self):
        if self.sync and self.training and dist.is_available() and dist.is_initialized() \
                and dist.get_world_size(self.process_group) > 1:
            return self.process_group if self.process_group is not None else dist.group.WORLD
        return None

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                residual_is_ancestor: bool = False, bn_stats=None, pool: Optional[nn.Module] = None,
                defer: bool = False) -> torch.Tensor:
        """``residual_is_ancestor``: the caller guarantees ``x`` is computed from
        ``residual`` (ResNet identity shortcut), so this layer's backward runs before
        the residual producer's and the residual gradient can be folded into it.
        ``bn_stats``: an ``ops.conv.BNStats`` the conv producing ``x`` may have filled
        with x's partial sums (this layer then skips its own partial pass).
        ``pool``: a max-pool module applied to this layer's output -- returns
        ``pool(self(x))``, on the training path as ONE pass (BatchNorm + ReLU folded
        into the pool kernel; the normalised activation is never materialised).
        ``defer``: the caller's only consumer of the output is a 1x1 conv that can apply
        this layer's map itself (:class:`DeferredApply`); honoured on the fused training
        path of a ReLU layer without residual or pool, else ignored."""
        geo = self._pool_geometry(pool, residual) if pool is not None else None
        if pool is not None and (geo is None or not fused_ok(x, residual)
                                 or not (self.training or not self.track_running_stats)):
            return pool(self.forward(x, residual, residual_is_ancestor, bn_stats))
        part = None
        if bn_stats is not None:
            part, bn_stats.part = bn_stats.part, None
        relu = self.act == "relu"
        use_batch_stats = self.training or not self.track_running_stats
        if fused_ok(x, residual):
            if use_batch_stats:
                stats["fused"] += 1
                track = self.training and self.track_running_stats
                momentum = -1.0 if self.momentum is None else float(self.momentum)
                slot = sink = None
                if self.fold_residual_grad and torch.is_grad_enabled():
                    slot = _FoldSlot()
                    src = getattr(residual, "_rla_fold", None) if residual is not None else None
                    if residual_is_ancestor and src is not None and not src.claimed and residual.requires_grad:
                        src.claimed, sink = True, src
                        residual = residual.detach()
                pre = None
                if defer and relu and residual is None and geo is None and defer_enabled():
                    pre = DeferredApply()
                    fold_stats["deferred"] += 1
                y = _BNActFn.apply(
                    x, self.weight, self.bias, residual,
                    self.running_mean if track else None, self.running_var if track else None,
                    self.num_batches_tracked if track else None, momentum, float(self.eps), relu, self._group(),
                    slot, sink, part, geo, pre)
                if slot is not None:
                    y._rla_fold = slot
                if pre is not None:
                    y._rla_pre = pre
                return y
            if not torch.is_grad_enabled() or not (x.requires_grad or (self.weight is not None
                                                                          and self.weight.requires_grad)):
                stats["fused"] += 1
                invstd = (self.running_var + self.eps).rsqrt()
                scale = invstd * self.weight if self.weight is not None else invstd
                shift = (self.bias if self.bias is not None else torch.zeros_like(invstd)) - self.running_mean * scale
                y = torch.empty_like(x, memory_format=torch.channels_last)
                require().bn_apply(_nhwc(x), scale.float().contiguous(), shift.float().contiguous(),
                                   _nhwc(residual) if residual is not None else None, relu, _nhwc(y))
                return y
        stats["fallback"] += 1
        if self._group() is not None and x.is_cuda:
            y = nn.SyncBatchNorm.forward(self, x)  # torch's cross-rank statistics
        else:
            if self._group() is not None and not self._warned:
                warnings.warn("BatchNormAct2d: synchronised statistics need GPU tensors; using local statistics")
                self._warned = True
            y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y


def convert_sync_batchnorm(module: nn.Module, process_group=None) -> nn.Module:
    """``nn.SyncBatchNorm.convert_sync_batchnorm`` that keeps fused BN+act layers
    fused (they switch to all-reduced statistics instead of being replaced)."""
    if isinstance(module, BatchNormAct2d):
        module.sync = True
        module.process_group = process_group
        return module
    if isinstance(module, nn.modules.batchnorm._BatchNorm) and not isinstance(module, nn.SyncBatchNorm):
        return nn.SyncBatchNorm.convert_sync_batchnorm(module, process_group)
    for name, child in list(module.named_children()):
        new = convert_sync_batchnorm(child, process_group)
        if new is not child:
            setattr(module, name, new)
    return module
