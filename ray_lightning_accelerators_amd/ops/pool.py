"""NHWC bf16 max pooling on the gfx950 kernels of ``csrc/pool.hip``.

``MaxPool2dNHWC`` is a drop-in ``nn.MaxPool2d`` for channels_last bf16
activations (ResNet-50's 3x3 / stride 2 stem pool under bf16 autocast): the
forward keeps a ONE-byte window argmax instead of PyTorch's int64 indices and
the backward gathers through it (no scatter, no atomics) -- PyTorch-ROCm's
``max_pool_backward_nhwc`` took 316 us per ResNet-50 step
(profiles/r1_resnet50_v2/kernel_stats_native_fusedbn.csv).  Ties and NaNs follow
PyTorch's rule, so the gradient is the same.  Other inputs (CPU, fp32, NCHW,
dilation, ceil_mode, C % 8 != 0) use ``F.max_pool2d``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import require, use_native


def _nhwc_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.size(1) % 8 == 0
            and x.permute(0, 2, 3, 1).is_contiguous() and x.data_ptr() % 16 == 0 and use_native(x))


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k: int, s: int, pad: int):
        y, arg = require().maxpool_fwd(x.permute(0, 2, 3, 1), k, s, pad)
        ctx.geom = (x.size(2), x.size(3), k, s, pad)
        ctx.save_for_backward(arg)
        ctx.mark_non_differentiable(arg)
        return y.permute(0, 3, 1, 2)  # NCHW logical shape, channels_last memory

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        H, W, k, s, pad = ctx.geom
        dyv = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        dx = require().maxpool_bwd(dyv, arg, H, W, k, s, pad)
        return dx.permute(0, 3, 1, 2), None, None, None


def max_pool2d_nhwc(x: torch.Tensor, kernel_size: int, stride: int, padding: int = 0) -> torch.Tensor:
    if _nhwc_ok(x) and 2 * padding <= kernel_size:
        return _MaxPoolFn.apply(x, int(kernel_size), int(stride), int(padding))
    return F.max_pool2d(x, kernel_size, stride, padding)


class MaxPool2dNHWC(nn.MaxPool2d):
    """``nn.MaxPool2d`` (square kernel / stride / padding, no dilation or ceil mode)
    with the fused NHWC bf16 path."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        k, s, p = self.kernel_size, self.stride, self.padding
        if (isinstance(k, int) and isinstance(s, int) and isinstance(p, int) and self.dilation == 1
                and not self.ceil_mode and not self.return_indices):
            return max_pool2d_nhwc(x, k, s, p)
        return super().forward(x)


class _GlobalAvgPoolFn(torch.autograd.Function):
    """[N, C, H, W] channels_last bf16 -> [N, C]: the mean over H*W (torch's reduce
    kernel), backward one gfx950 broadcast-store kernel straight into channels_last
    memory (``gap_bwd``)."""

    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        ctx.geom = (n, c, h, w)
        return x.permute(0, 2, 3, 1).reshape(n, h * w, c).mean(1)

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w = ctx.geom
        dx = require().gap_bwd(dy.to(torch.bfloat16).contiguous(), h * w)
        return dx.view(n, h, w, c).permute(0, 3, 1, 2)


def global_avg_pool_nhwc(x: torch.Tensor) -> torch.Tensor:
    """``torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)`` with the NHWC backward kernel."""
    if _nhwc_ok(x):
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
