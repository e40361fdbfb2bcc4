"""bf16 weight shadows for bf16 compute on fp32 master weights.

Under bf16 autocast every convolution casts its fp32 weight to bf16 in every
forward (ResNet-50: 56 small cast kernels, ~260 us a step,
profiles/r3_rn50/kernel_stats_rn50_steady.csv).  When the parameters live in a
:class:`~ray_lightning_accelerators_amd.parallel.arena.ParamArena` with a bf16
shadow, the fused optimizer step writes the bf16 copy in the same pass as the
fp32 update, and the shadow-aware layers here read it directly; the gradient
still reaches the fp32 parameter (the backward's bf16 -> fp32 conversion is the
one autocast performs too).
"""
from __future__ import annotations

import weakref
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

_arenas: "weakref.WeakSet" = weakref.WeakSet()
stats = {"shadow": 0, "cast": 0}


def register(arena) -> None:
    _arenas.add(arena)


def bf16_weight(p: torch.Tensor) -> Optional[torch.Tensor]:
    for a in list(_arenas):
        w = a.bf16_weight(p)
        if w is not None:
            return w
    return None


def wants_shadow(module: nn.Module) -> bool:
    """True when the module has layers that read bf16 shadows."""
    return any(getattr(m, "_rla_reads_bf16_shadow", False) for m in module.modules())


class _ShadowWeight(torch.autograd.Function):
    """Forward: the bf16 shadow; backward: its gradient, in fp32, to the master weight."""

    @staticmethod
    def forward(ctx, weight, shadow):
        return shadow.view_as(shadow)

    @staticmethod
    def backward(ctx, g):
        return g.float(), None


def bf16_param(p: torch.Tensor) -> Optional[torch.Tensor]:
    """bf16 stand-in for ``p`` inside an autocast region (None: let autocast cast)."""
    w = bf16_weight(p)
    if w is None:
        stats["cast"] += 1
        return None
    stats["shadow"] += 1
    return _ShadowWeight.apply(p, w) if torch.is_grad_enabled() and p.requires_grad else w


class ConvBF16(nn.Conv2d):
    """``nn.Conv2d`` that, under CUDA bf16 autocast, convolves with the weight's bf16
    shadow instead of casting it (same parameters / state-dict keys)."""

    _rla_reads_bf16_shadow = True

    def forward(self, x: torch.Tensor, fork=None, bn_stats=None) -> torch.Tensor:
        """``fork``: an ops.conv.GradFork shared with another consumer of ``x`` (fast path only).
        ``bn_stats``: an ops.conv.BNStats the 3x3 MFMA forward may fill (the next
        BatchNorm's batch statistics from its epilogue)."""
        if getattr(x, "_rla_pre", None) is not None:
            # a deferred BatchNorm + ReLU output (ops/bn.py DeferredApply): only conv_nhwc
            # understands it -- every other path gets the materialised activation
            from .conv import kxk_fast_ok
            from .bn import materialize

            wb = bf16_weight(self.weight)
            if not (x.is_cuda and torch.is_autocast_enabled("cuda") and self.padding_mode == "zeros"
                    and wb is not None and torch.is_grad_enabled() and self.weight.requires_grad
                    and kxk_fast_ok(x, self)):
                x = materialize(x)
        if x.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16 \
                and self.padding_mode == "zeros":
            wb = bf16_weight(self.weight)
            if wb is not None and torch.is_grad_enabled() and self.weight.requires_grad:
                from .conv import conv_nhwc, kxk_fast_ok, stem_conv, stem_fast_ok

                xb = x.to(torch.bfloat16)
                if stem_fast_ok(xb, self):
                    # ResNet stem: MFMA kernel (+ the next BatchNorm's statistics)
                    stats["shadow"] += 1
                    return stem_conv(xb, self, wb, bn_stats)
                if kxk_fast_ok(xb, self):
                    # MIOpen forward / dgrad, weight gradient from the MFMA kernel when
                    # it is the faster one (ops/conv.py)
                    stats["shadow"] += 1
                    return conv_nhwc(xb, self, wb, fork, bn_stats)
            w = bf16_param(self.weight)
            if w is not None:
                b = self.bias.to(torch.bfloat16) if self.bias is not None else None
                return F.conv2d(x.to(torch.bfloat16), w, b, self.stride, self.padding, self.dilation, self.groups)
        return super().forward(x)
