"""Stride-1 1x1 convolution on NHWC bf16 activations, backend chosen per operation.

A 1x1 convolution over a channels_last tensor IS a GEMM on the [N*H*W, C] view:

  forward  y[M, Cout]  = x[M, Cin]  . W^T
  dgrad    dx[M, Cin]  = dy[M, Cout] . W
  wgrad    dW[Cout, Cin] = dy^T . x      (fp32 output: the fp32 master gradient)

MIOpen runs these as convolutions; for ResNet-50's shapes it is the faster choice
for some (e.g. the wgrad of the large 56x56 layers) and far slower for others: its
wgrad costs ~80 us whatever the size (zero-fill + split-K atomics + a bf16->fp32
cast, profiles/r3_rn50/kernel_stats_rn50_steady.csv) and its forward of the
14x14 / 7x7 layers runs 2-5x a hipBLASLt GEMM (profiles/r3_rn50/conv1x1_probe_perop.log).
So every (operation, shape) picks its backend once, timed on the device at first
use (like cudnn.benchmark), and the GEMM wgrad writes fp32 directly -- no zero
fill, no atomics, no cast kernel.

``Conv1x1NHWC`` is a drop-in ``nn.Conv2d(cin, cout, 1, bias=False)`` (same
parameter and state-dict key); anything outside the fast path (CPU, fp32, NCHW,
odd alignment) runs the stock convolution.  ``RLA_CONV1X1=miopen|gemm|auto``.
"""
from __future__ import annotations

import functools
import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

_choice: Dict[Tuple[str, int, int, int], str] = {}
_timings: Dict[Tuple[str, int, int, int], Dict[str, float]] = {}
stats = {"fast": 0, "fallback": 0, "bn_dgrad_fused": 0, "stem": 0, "pre_applied": 0}

_conv = torch.ops.aten.convolution
_conv_bwd = torch.ops.aten.convolution_backward


def _mode() -> str:
    return os.environ.get("RLA_CONV1X1", "auto")


def _wmode() -> str:
    """``RLA_CONV_WGRAD``: backend of the weight gradients (auto: timed per shape)."""
    return os.environ.get("RLA_CONV_WGRAD", "auto")


_REPS = 3
_DETERMINISTIC_ORDER = ("hip", "hip_gen", "gemm", "miopen")


def _time(fn, reps: int = _REPS) -> float:
    """Device time of ``reps`` calls.  The device is held by a spin kernel while the
    host enqueues them, so the calls run back to back: a backend's host-side cost
    (MIOpen's is tens of us per call) is hidden, as it is inside a GPU-bound step --
    timing an idle device would charge it to the kernels."""
    fn()  # warm: library kernel load / solver search
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def _pick(op: str, key: Tuple[int, ...], cands) -> str:
    mode = _mode()
    if op.startswith("wgrad"):
        # RLA_CONV_WGRAD picks the weight-gradient backend; RLA_CONV1X1=miopen|gemm
        # still pins the 1x1 layers' wgrad when it is left on auto
        mode = _wmode() if _wmode() != "auto" or op != "wgrad" else mode
    if mode in cands:
        return mode
    if torch.are_deterministic_algorithms_enabled():
        # Trainer(deterministic=True): no timing (two runs could pick different
        # kernels that round differently), and never MIOpen's split-K-atomic wgrad:
        # the MFMA kernel (fixed-order split reduction), else the GEMM
        for name in _DETERMINISTIC_ORDER:
            if name in cands:
                return name
    k = (op,) + key
    c = _choice.get(k)
    if c is None and torch.cuda.is_current_stream_capturing():
        return "miopen"  # no timing inside a graph capture (it synchronises)
    if c is None:
        # two rounds, each candidate's best: one noisy window (MIOpen's first calls
        # of a shape vary by 2x on a fresh box) must not decide the backend
        t = {name: _time(fn, _REPS) for name, fn in cands.items()}
        for name, fn in cands.items():
            t[name] = min(t[name], _time(fn, _REPS))
        c = min(t, key=t.get)
        _choice[k] = c
        _timings[k] = {name: round(v * 1e3 / _REPS, 1) for name, v in t.items()}  # device us per call
    return c


def choices() -> Dict[str, Dict[str, float]]:
    """The autotuned backends so far: ``"op M Cin Cout" -> {backend: us, ..., "pick": name}``."""
    return {" ".join(map(str, k)): dict(_timings.get(k, {}), pick=c) for k, c in _choice.items()}


def wgrad_ok(cin: int, cout: int) -> bool:
    """Shapes the MFMA weight-gradient kernel covers (csrc/conv_wgrad.hip)."""
    return cin % 64 == 0 and cout % 64 == 0 and os.environ.get("RLA_CONV_WGRAD", "auto") != "off"


def wgrad_hip(dy: torch.Tensor, x: torch.Tensor, kernel_size, stride, padding, splits: int = 0,
              algo: int = 0, pre_ss: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weight gradient of an NHWC bf16 convolution on the MFMA kernel: ``dy`` [N, Cout,
    OH, OW] and ``x`` [N, Cin, H, W], both channels_last bf16; returns the fp32
    gradient [Cout, Cin, KH, KW] with channels_last strides (the kernel writes the
    [Cout, KH, KW, Cin] memory order directly).  ``algo`` 0: the 3x3 / stride-1 /
    pad-1 halo kernel where it applies, else the generic one; 1: always generic.
    ``pre_ss`` (1x1 / stride 1): ``x`` is a deferred BatchNorm + ReLU's input and the
    kernel stages relu(x * scale + shift) (ops/bn.py DeferredApply)."""
    from . import require

    n, cin, h, w = x.shape
    cout, oh, ow = dy.size(1), dy.size(2), dy.size(3)
    kh, kw = kernel_size
    out = require().conv_wgrad(dy.permute(0, 2, 3, 1), x.permute(0, 2, 3, 1), n, h, w, cin, oh, ow, cout, kh, kw,
                               stride[0], stride[1], padding[0], padding[1], splits, algo, pre_ss)
    return out.permute(0, 3, 1, 2)


def conv3x3_ok(x: torch.Tensor, wb: torch.Tensor, stride, padding) -> bool:
    """3x3 / stride 1 / pad 1 layers the MFMA convolution kernel covers (csrc/conv3x3.hip)."""
    if tuple(wb.shape[2:]) != (3, 3) or tuple(stride) != (1, 1) or tuple(padding) != (1, 1):
        return False
    if os.environ.get("RLA_CONV3X3", "auto") == "off":
        return False
    n, cin, h, w = x.shape
    cout = wb.size(0)
    return (cin % 64 == 0 and cout % 64 == 0 and wb.is_contiguous(memory_format=torch.channels_last)
            and _conv3x3_shape_ok(n, h, w, cin, cout))


@functools.lru_cache(maxsize=256)
def _bn_bwd_shape_ok(m: int, k: int, n: int) -> bool:
    from . import require

    return bool(require().conv1x1_bn_bwd_ok(m, k, n))


@functools.lru_cache(maxsize=256)
def _conv3x3_shape_ok(n: int, h: int, w: int, cin: int, cout: int) -> bool:
    from . import require

    return bool(require().conv3x3_supported(n, h, w, cin, cout))


def conv3x3_hip(x: torch.Tensor, wb: torch.Tensor) -> torch.Tensor:
    """``conv2d(x, wb, stride=1, padding=1)`` on the MFMA kernel: ``x`` [N, Cin, H, W]
    channels_last bf16, ``wb`` [Cout, Cin, 3, 3] channels_last bf16 (its memory IS the
    kernel's [Cout][3][3][Cin]); returns [N, Cout, H, W] channels_last."""
    from . import require

    n, cin, h, w = x.shape
    cout = wb.size(0)
    y = require().conv3x3(x.permute(0, 2, 3, 1), wb.permute(0, 2, 3, 1), n, h, w, cin, cout)
    return y.permute(0, 3, 1, 2)


def conv3x3_stats_hip(x: torch.Tensor, wb: torch.Tensor, pre=None):
    """:func:`conv3x3_hip` plus the per-channel partial sums of its bf16 output from the
    epilogue (csrc/conv3x3.hip ST): returns (y channels_last, part [rows, 2, Cout]).
    ``pre`` (ops/bn.py DeferredApply): ``x`` is that BatchNorm's input and the kernel
    convolves relu(x * scale + shift), with zero padding (csrc/conv3x3.hip PRE)."""
    from . import require

    n, cin, h, w = x.shape
    cout = wb.size(0)
    if pre is not None:
        y, part = require().conv3x3_stats(x.permute(0, 2, 3, 1), wb.permute(0, 2, 3, 1), n, h, w, cin, cout,
                                          pre.st, pre.take_nbt())
    else:
        y, part = require().conv3x3_stats(x.permute(0, 2, 3, 1), wb.permute(0, 2, 3, 1), n, h, w, cin, cout)
    return y.permute(0, 3, 1, 2), part


class _TimingPre:
    """A DeferredApply stand-in for timing candidates: same statistics, no
    num_batches_tracked increment."""

    __slots__ = ("st",)

    def __init__(self, pre):
        self.st = pre.st

    def take_nbt(self):
        return None


def _applied(x: torch.Tensor, pre) -> torch.Tensor:
    """relu(x * scale + shift) by the apply kernel (a timing candidate: no autograd)."""
    from . import require

    y = torch.empty_like(x, memory_format=torch.channels_last)
    require().bn_apply(x.permute(0, 2, 3, 1), pre.st[2], pre.st[3], None, True, y.permute(0, 2, 3, 1))
    return y


def conv3x3_stats_enabled() -> bool:
    """``RLA_CONV3X3_STATS=off`` keeps the 3x3 forward's BatchNorm statistics in BN's own pass."""
    return os.environ.get("RLA_CONV3X3_STATS", "auto") != "off"


def conv3x3_dgrad_hip(dy: torch.Tensor, wb: torch.Tensor) -> torch.Tensor:
    """Input gradient of a 3x3 / stride 1 / pad 1 convolution = the same convolution
    of ``dy`` with the weight flipped in both taps and transposed in channels; the
    kernel reads the forward weight that way itself (no re-layout kernel)."""
    from . import require

    n, cout, h, w = dy.shape
    cin = wb.size(1)
    dx = require().conv3x3(dy.permute(0, 2, 3, 1), wb.permute(0, 2, 3, 1), n, h, w, cout, cin, True)
    return dx.permute(0, 3, 1, 2)


def _nhwc2d(t: torch.Tensor) -> torch.Tensor:
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _from2d(t2: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return t2.view(n, h, w, t2.size(1)).permute(0, 3, 1, 2)


class GradFork:
    """Two convolutions reading the SAME input (a bottleneck's conv1 and its
    downsample conv): their input gradients meet in ONE tensor instead of two
    tensors and an autograd add kernel (``CUDAFunctor_add<bf16>``,
    ~200 us per ResNet-50 step).  Whichever backward runs first parks its full dgrad
    here and returns None for the input; the second accumulates its contribution
    INTO that tensor -- a GEMM with beta = 1 (stride 1), or a GEMM on the
    subsampled rows plus an add into every s-th pixel only (stride s > 1) -- and
    returns the sum.  Order-independent; autograd sees None + sum.  Only when BOTH
    consumers took a fast path (each registers in its forward): with one consumer on a
    stock fallback, the fast one returns its own gradient and autograd adds as usual."""

    __slots__ = ("dx", "users")

    def __init__(self):
        self.dx: Optional[torch.Tensor] = None
        self.users = 0


def _fork_dx(fork: Optional[GradFork], full, accumulate) -> Optional[torch.Tensor]:
    """``full()``: this op's dgrad as a new tensor; ``accumulate(d)``: add it into ``d``."""
    if fork is None or fork.users < 2:
        return full()
    if fork.dx is None:
        fork.dx = full()
        return None
    d, fork.dx = fork.dx, None
    if accumulate is None:
        d.add_(full())  # no fused form for this op: a plain add (still one tensor less)
    else:
        accumulate(d)
    return d


def _acc_dgrad(d: torch.Tensor, dy2: torch.Tensor, wb: torch.Tensor) -> None:
    """d += dy . W for a stride-1 1x1 conv: in the GEMM (beta = 1) on d's NHWC view."""
    if d.permute(0, 2, 3, 1).is_contiguous():
        _nhwc2d(d).addmm_(dy2, wb)
    else:
        d.add_(_from2d(torch.mm(dy2, wb), d.size(0), d.size(2), d.size(3)))


class BNStats:
    """Hand-off of a convolution's epilogue BatchNorm statistics to the BatchNorm that
    consumes its output: the conv fills ``part`` ([rows, 2, C] fp32 partial sums of
    its bf16 output, ``bn_finalize``'s layout) when its backend computed them, and
    ``BatchNormAct2d`` then skips its own partial pass over the output."""

    __slots__ = ("part",)

    def __init__(self):
        self.part: Optional[torch.Tensor] = None


def conv1x1_stats_ok(m: int, cin: int, cout: int) -> bool:
    """Shapes of the 1x1 MFMA forward with BatchNorm statistics (csrc/conv1x1.hip)."""
    return cin % 32 == 0 and cout % 64 == 0 and cout <= 4096 and os.environ.get("RLA_CONV1X1_STATS", "auto") != "off"


def conv1x1_stats_hip(x: torch.Tensor, wb: torch.Tensor, pre=None):
    """``conv2d(x, wb)`` for a 1x1 / stride-1 layer on the MFMA kernel, plus the
    per-channel partial sums of its bf16 output: ``x`` [N, Cin, H, W] channels_last
    bf16, ``wb`` [Cout, Cin] bf16.  Returns (y channels_last, part [rows, 2, Cout]).
    ``pre`` (ops/bn.py DeferredApply): ``x`` is that BatchNorm's input and the kernel
    convolves relu(x * scale + shift) instead."""
    from . import require

    n, _, h, w = x.shape
    if pre is not None:
        y2, part = require().conv1x1_stats(_nhwc2d(x), wb, pre.st, pre.take_nbt())
    else:
        y2, part = require().conv1x1_stats(_nhwc2d(x), wb)
    return _from2d(y2, n, h, w), part


def conv1x1_pre_ok(m: int, cin: int, cout: int) -> bool:
    """Where a 1x1 conv applies a deferred BatchNorm + ReLU in its own kernels (forward
    and weight gradient): K <= 128, the shapes whose forward runs on the in-tree kernel
    anyway (profiles/r5_pair/rn50_graph.log ``fwd_st``; at K >= 256 the library GEMM +
    the apply pass is faster)."""
    return cin <= 128 and conv1x1_stats_ok(m, cin, cout) and wgrad_ok(cin, cout)


def fuse_bn_dgrad_enabled() -> bool:
    """A 1x1 conv marked ``fuse_bn_dgrad`` (ResNet's identity-block conv1, whose input
    y is a residual BatchNorm+ReLU's output with no other autograd consumer: the
    identity shortcut's gradient is folded) computes that BatchNorm's backward partial
    in its input-gradient kernel (csrc/conv1x1.hip BWD): d = (dx + dy2) * (y > 0) is
    written once and the plain input gradient is never materialised.
    ``RLA_FUSE_BN_DGRAD=0`` turns it off (same-box A/B: +0.5 %, profiles/r4_c1)."""
    return os.environ.get("RLA_FUSE_BN_DGRAD", "1") == "1"


def _bn_partial(y: torch.Tensor) -> torch.Tensor:
    from . import require

    return require().bn_partial(y.permute(0, 2, 3, 1), None, None, y.size(1), 0, False, None)


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, shadow=None, fork=None, bn_stats=None, fuse_bn=False, pre=None):
        n, cin, h, w = x.shape
        cout = weight.size(0)
        # the arena's bf16 shadow (ops/shadow.py) when there is one: no cast kernel
        wb = (shadow if shadow is not None else weight.detach().to(torch.bfloat16)).reshape(cout, cin)
        x2 = _nhwc2d(x)
        key = (x2.size(0), cin, cout)
        w4 = wb.view(cout, cin, 1, 1)
        ctx.pre_st = None
        if pre is not None:
            # x is a deferred BatchNorm + ReLU's input (ops/bn.py DeferredApply): the
            # kernels apply its map to their operands; the caller checked conv1x1_pre_ok
            y, part = conv1x1_stats_hip(x, wb, pre)
            if bn_stats is not None:
                bn_stats.part = part
            ctx.pre_st = pre.st
            ctx.save_for_backward(x, wb)
            ctx.key, ctx.fork, ctx.fold = key, None, None
            return y
        if bn_stats is not None and conv1x1_stats_ok(x2.size(0), cin, cout):
            # the next BatchNorm's statistics: in this GEMM's epilogue, or the library
            # forward + BN's own partial pass -- whichever is faster for the shape
            be = _pick("fwd_st", key, {
                "hip": lambda: conv1x1_stats_hip(x, wb),
                "gemm": lambda: _bn_partial(_from2d(torch.mm(x2, wb.t()), n, h, w)),
                "miopen": lambda: _bn_partial(_conv(x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)),
            })
        else:
            be = _pick("fwd", key, {
                "gemm": lambda: torch.mm(x2, wb.t()),
                "miopen": lambda: _conv(x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1),
            })
        if be == "hip":
            y, bn_stats.part = conv1x1_stats_hip(x, wb)
        elif be == "gemm":
            y = _from2d(torch.mm(x2, wb.t()), n, h, w)
        else:
            y = _conv(x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        ctx.save_for_backward(x, wb)
        ctx.key = key
        ctx.fork = fork
        if fork is not None:
            fork.users += 1
        # x is a residual BatchNorm+ReLU's output (its fold slot carries that layer's
        # input): the input gradient may absorb the BatchNorm's backward partial
        fold = getattr(x, "_rla_fold", None)
        ctx.fold = fold if (fuse_bn and fork is None and fold is not None and getattr(fold, "x3", None) is not None
                            and fuse_bn_dgrad_enabled()
                            and _bn_bwd_shape_ok(x2.size(0), cout, cin)) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        n, cin, h, w = x.shape
        cout = wb.size(0)
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy2, x2 = _nhwc2d(dy), _nhwc2d(x)
        w4 = wb.view(cout, cin, 1, 1)
        dx = dw = None
        be_d = be_w = None
        fork = ctx.fork if ctx.needs_input_grad[0] else None
        fold = ctx.fold
        if ctx.pre_st is not None:
            # deferred-BatchNorm input: the input gradient (w.r.t. the activation) does not
            # read x; the weight gradient stages relu(x * scale + shift) in its kernel
            if ctx.needs_input_grad[0]:
                be_d = _pick("dgrad", ctx.key, {
                    "gemm": lambda: torch.mm(dy2, wb),
                    "miopen": lambda: _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                [True, False, False])[0],
                })
                if be_d == "gemm":
                    dx = _from2d(torch.mm(dy2, wb), n, h, w)
                else:
                    dx = _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0]
            if ctx.needs_input_grad[1]:
                dw = wgrad_hip(dy, x, (1, 1), (1, 1), (0, 0), pre_ss=ctx.pre_st)
            return dx, dw, None, None, None, None, None
        if fold is not None and fold.dres is not None and ctx.needs_input_grad[0]:
            # d = (dy . W + dres_next) * (x > 0) and its BatchNorm partial sums in one
            # kernel; the producer BatchNorm's backward takes d as its dy
            from . import require
            from .bn import fold_stats

            d2, part = require().conv1x1_bn_bwd(dy2, wb.t().contiguous(), _nhwc2d(fold.dres), x2,
                                                _nhwc2d(fold.x3))
            fold.dres, fold.bwd_part = None, part
            fold_stats["folded"] += 1
            stats["bn_dgrad_fused"] += 1
            dx = _from2d(d2, n, h, w)
            fold.bwd_d = dx  # bn backward checks it receives exactly this tensor
        elif fork is not None and fork.users >= 2 and fork.dx is not None:
            # second of a forked pair: dx += dy . W in the GEMM itself (beta = 1)
            dx = _fork_dx(fork, None, lambda d: _acc_dgrad(d, dy2, wb))
        elif ctx.needs_input_grad[0]:
            be_d = _pick("dgrad", ctx.key, {
                "gemm": lambda: torch.mm(dy2, wb),
                "miopen": lambda: _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                            [True, False, False]),
            })
        if ctx.needs_input_grad[1]:
            cands = {
                "gemm": lambda: torch.ops.aten.mm.dtype(dy2.t(), x2, torch.float32),
                "miopen": lambda: _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                            [False, True, False])[1].float(),
            }
            if wgrad_ok(cin, cout):
                cands["hip"] = lambda: wgrad_hip(dy, x, (1, 1), (1, 1), (0, 0))
            be_w = _pick("wgrad", ctx.key, cands)
        if be_d == "miopen" and be_w == "miopen" and fork is None:
            # both from MIOpen: one call (its host cost is tens of us per call)
            dx, dw = _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, True, False])[:2]
            return dx, dw.float(), None, None, None, None, None
        if be_d == "gemm":
            dx = _fork_dx(fork, lambda: _from2d(torch.mm(dy2, wb), n, h, w), None)
        elif be_d == "miopen":
            dx = _fork_dx(fork, lambda: _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                  [True, False, False])[0], None)
        if be_w == "hip":
            dw = wgrad_hip(dy, x, (1, 1), (1, 1), (0, 0))
        elif be_w == "gemm":
            dw = torch.ops.aten.mm.dtype(dy2.t(), x2, torch.float32).view(cout, cin, 1, 1)
        elif be_w == "miopen":
            dw = _conv_bwd(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                           [False, True, False])[1].float()
        return dx, dw, None, None, None, None, None


def fast_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.numel() > 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
            and conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.padding == (0, 0)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and x.size(1) % 8 == 0 and conv.out_channels % 8 == 0)


class Conv1x1NHWC(nn.Conv2d):
    """``nn.Conv2d(cin, cout, 1, bias=False)`` with per-operation MIOpen / GEMM backends."""

    _rla_reads_bf16_shadow = True

    def __init__(self, in_channels: int, out_channels: int, device=None, dtype=None):
        super().__init__(in_channels, out_channels, 1, 1, 0, bias=False, device=device, dtype=dtype)
        # set by a model whose structure makes this layer its input's only autograd
        # consumer (see fuse_bn_dgrad_enabled)
        self.fuse_bn_dgrad = False

    def forward(self, x: torch.Tensor, fork: Optional[GradFork] = None,
                bn_stats: Optional[BNStats] = None) -> torch.Tensor:
        """``bn_stats``: the BatchNorm reading this output is training on batch
        statistics -- let this layer compute them where that is faster (BNStats)."""
        pre = getattr(x, "_rla_pre", None)
        if pre is not None:
            # a deferred BatchNorm + ReLU output (ops/bn.py DeferredApply): applied in this
            # conv's kernels where the shape allows, else materialised here
            from .bn import materialize

            if (fork is None and fast_ok(x, self) and _mode() != "off" and not pre.used
                    and conv1x1_pre_ok(x.size(0) * x.size(2) * x.size(3), x.size(1), self.out_channels)):
                pre.used = True
                stats["fast"] += 1
                stats["pre_applied"] += 1
                from .shadow import bf16_weight

                return _Conv1x1Fn.apply(x, self.weight, bf16_weight(self.weight), None, bn_stats, False, pre)
            x = materialize(x)
        if torch.is_autocast_enabled("cuda") and x.is_cuda and x.dtype == torch.float32:
            x = x.to(torch.bfloat16)
        if fast_ok(x, self) and _mode() != "off":
            stats["fast"] += 1
            from .shadow import bf16_weight

            return _Conv1x1Fn.apply(x, self.weight, bf16_weight(self.weight), fork, bn_stats, self.fuse_bn_dgrad)
        stats["fallback"] += 1
        return F.conv2d(x, self.weight)


class _ConvNHWCFn(torch.autograd.Function):
    """KxK (or strided) bf16 NHWC convolution: MIOpen forward and dgrad, the weight
    gradient from MIOpen or the MFMA kernel (``wgrad_hip``), picked per shape on
    device time.  The weight gradient reaches the fp32 master weight in fp32."""

    @staticmethod
    def forward(ctx, x, weight, wb, stride, padding, fork=None, bn_stats=None, pre=None):
        ctx.pre_st = None
        if pre is not None:
            # x is a deferred BatchNorm + ReLU's input (ops/bn.py DeferredApply): the
            # forward stages the activation itself (conv_nhwc chose this path)
            y, bn_stats.part = conv3x3_stats_hip(x, wb, pre)
            ctx.pre_st = pre.st
            ctx.c3 = True
            ctx.save_for_backward(x, wb)
            ctx.geo = (tuple(stride), tuple(padding))
            ctx.fork = None
            return y
        ctx.c3 = conv3x3_ok(x, wb, stride, padding)
        be = "miopen"
        if ctx.c3:
            key = (x.size(0) * x.size(2) * x.size(3), x.size(1), wb.size(0), 3, 3, 1, 1)
            if bn_stats is not None and conv3x3_stats_enabled():
                # the next BatchNorm's statistics: in this kernel's epilogue, or the
                # library forward + BN's own partial pass -- whichever is faster
                be = _pick("fwd_kxk_st", key, {
                    "miopen": lambda: _bn_partial(_conv(x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1)),
                    "hip_st": lambda: conv3x3_stats_hip(x, wb),
                })
            else:
                be = _pick("fwd_kxk", key, {
                    "miopen": lambda: _conv(x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1),
                    "hip": lambda: conv3x3_hip(x, wb),
                })
        if be == "hip_st":
            y, bn_stats.part = conv3x3_stats_hip(x, wb)
        elif be == "hip":
            y = conv3x3_hip(x, wb)
        else:
            y = _conv(x, wb, None, list(stride), list(padding), [1, 1], False, [0, 0], 1)
        ctx.save_for_backward(x, wb)
        ctx.geo = (tuple(stride), tuple(padding))
        ctx.fork = fork
        if fork is not None:
            fork.users += 1
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        stride, padding = ctx.geo
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        be = None
        fork = ctx.fork if ctx.needs_input_grad[0] else None
        if fork is not None and fork.users >= 2 and fork.dx is not None and wb.shape[2:] == (1, 1) \
                and padding == (0, 0):
            # second of a forked pair, strided 1x1: GEMM over the output pixels, added
            # into every stride-th input pixel of the parked dgrad (1/s^2 of it)
            cout, cin = wb.shape[:2]
            n_, _, oh_, ow_ = dy.shape
            w2 = wb.reshape(cout, cin)

            g2 = torch.mm(_nhwc2d(dy), w2)

            def acc(d):
                # (measured and reverted, round 5: the same sum as ONE strided batched
                # GEMM with beta = 1 into every stride-th pixel -- hipBLASLt ran it as
                # MT256x16x64 at ~205 us a call vs ~21 us for this GEMM + strided add)
                s_ = stride[0]
                if (s_ == stride[1] and d.dtype == torch.bfloat16 and g2.dtype == torch.bfloat16
                        and d.is_contiguous(memory_format=torch.channels_last) and g2.is_contiguous()
                        and d.size(1) % 8 == 0 and (d.size(2) - 1) // s_ + 1 == oh_
                        and (d.size(3) - 1) // s_ + 1 == ow_):
                    # 16-byte vectors over the NHWC rows, same fp32 add + one rounding
                    # as ATen's add_ (which took its non-vectorised strided path)
                    from . import require

                    require().strided_add_(d, g2, s_)
                    return
                view = d[:, :, ::stride[0], ::stride[1]]
                view.add_(_from2d(g2, n_, oh_, ow_))

            dx = _fork_dx(fork, None, acc)
            fork = None  # the input gradient is settled
        if ctx.pre_st is not None:
            # deferred-BatchNorm input: the weight gradient stages relu(x * scale + shift)
            # (halo or generic MFMA kernel, csrc/conv_wgrad.hip PRE); the input gradient
            # does not read x
            cout, cin, kh, kw = wb.shape
            if ctx.needs_input_grad[1]:
                key = (x.size(0) * dy.size(2) * dy.size(3), cin, cout, kh, kw, stride[0], padding[0])
                st = ctx.pre_st
                bw = _pick("wgrad_kxk_pre", key, {
                    "hip": lambda: wgrad_hip(dy, x, (kh, kw), stride, padding, pre_ss=st),
                    "hip_gen": lambda: wgrad_hip(dy, x, (kh, kw), stride, padding, algo=1, pre_ss=st),
                })
                dw = wgrad_hip(dy, x, (kh, kw), stride, padding, algo=0 if bw == "hip" else 1, pre_ss=st)
            if ctx.needs_input_grad[0]:
                key = (x.size(0) * x.size(2) * x.size(3), cin, cout, 3, 3, 1, 1)
                be_d = _pick("dgrad_kxk", key, {
                    "miopen": lambda: _conv_bwd(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                [True, False, False])[0],
                    "hip": lambda: conv3x3_dgrad_hip(dy, wb),
                })
                if be_d == "hip":
                    dx = conv3x3_dgrad_hip(dy, wb)
                else:
                    dx = _conv_bwd(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0]
            return dx, dw, None, None, None, None, None, None
        if ctx.needs_input_grad[1]:
            cout, cin, kh, kw = wb.shape
            key = (x.size(0) * dy.size(2) * dy.size(3), cin, cout, kh, kw, stride[0], padding[0])
            cands = {
                "miopen": lambda: _conv_bwd(dy, x, wb, None, list(stride), list(padding), [1, 1], False, [0, 0], 1,
                                            [False, True, False])[1].float(),
                "hip": lambda: wgrad_hip(dy, x, (kh, kw), stride, padding),
            }
            if (kh, kw, tuple(stride), tuple(padding)) == (3, 3, (1, 1), (1, 1)):
                # "hip" is the halo kernel here; the generic tap-GEMM kernel competes too
                cands["hip_gen"] = lambda: wgrad_hip(dy, x, (kh, kw), stride, padding, algo=1)
            be = _pick("wgrad_kxk", key, cands)
        need_dx = bool(ctx.needs_input_grad[0]) and dx is None
        be_d = None
        if need_dx and ctx.c3:
            cout, cin = wb.shape[:2]
            key = (x.size(0) * x.size(2) * x.size(3), cin, cout, 3, 3, 1, 1)
            be_d = _pick("dgrad_kxk", key, {
                "miopen": lambda: _conv_bwd(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                            [True, False, False])[0],
                "hip": lambda: conv3x3_dgrad_hip(dy, wb),
            })
        if be_d == "hip":
            dx = _fork_dx(fork, lambda: conv3x3_dgrad_hip(dy, wb), None)
            need_dx = False
        if be == "miopen":
            # MIOpen for both gradients: one call, as F.conv2d's autograd makes it
            mask = [need_dx, True, False]
            dxm, dw = _conv_bwd(dy, x, wb, None, list(stride), list(padding), [1, 1], False, [0, 0], 1, mask)[:2]
            if need_dx:
                dx = _fork_dx(fork, lambda: dxm, None)
            return dx, dw.float(), None, None, None, None, None, None
        if need_dx:
            dx = _fork_dx(fork, lambda: _conv_bwd(dy, x, wb, None, list(stride), list(padding), [1, 1], False,
                                                  [0, 0], 1, [True, False, False])[0], None)
        if be == "hip":
            dw = wgrad_hip(dy, x, (kh, kw), stride, padding)
        elif be == "hip_gen":
            dw = wgrad_hip(dy, x, (kh, kw), stride, padding, algo=1)
        return dx, dw, None, None, None, None, None, None


@functools.lru_cache(maxsize=64)
def _stem_shape_ok(n: int, h: int, w: int) -> bool:
    from . import require

    return bool(require().stem_supported(n, h, w))


def stem_fast_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """The ResNet stem (7x7 / stride 2 / pad 3, 3 -> 64, no bias) on an NHWC bf16 input
    the MFMA stem kernel covers (csrc/stem.hip); ``RLA_STEM=off`` keeps MIOpen."""
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.size(1) == 3
            and conv.in_channels == 3 and conv.out_channels == 64 and conv.kernel_size == (7, 7)
            and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.dilation == (1, 1)
            and conv.groups == 1 and conv.bias is None and conv.padding_mode == "zeros"
            and os.environ.get("RLA_STEM", "auto") != "off" and _stem_shape_ok(x.size(0), x.size(2), x.size(3)))


def stem_hip(x: torch.Tensor, wb: torch.Tensor, stats: bool = False):
    """``conv2d(x, wb, stride=2, padding=3)`` for the stem on the MFMA kernel: ``x`` [N, 3,
    H, W] bf16 (any layout; made NHWC-contiguous), ``wb`` [64, 3, 7, 7] bf16 channels_last.
    Returns y [N, 64, OH, OW] channels_last, or (y, part [rows, 2, 64]) with ``stats``."""
    from . import require

    xn = x.permute(0, 2, 3, 1).contiguous()
    out = require().stem_fwd(xn, wb.permute(0, 2, 3, 1).contiguous(), stats)
    y = out[0].permute(0, 3, 1, 2)
    return (y, out[1]) if stats else y


def stem_wgrad_hip(x: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """Weight gradient of the stem on the MFMA kernel (csrc/stem.hip): fp32 [64, 3, 7, 7]
    with channels_last strides (the master weight's layout)."""
    from . import require

    dw = require().stem_wgrad(x.permute(0, 2, 3, 1).contiguous(), dy.permute(0, 2, 3, 1).contiguous())
    return dw.permute(0, 3, 1, 2)


class _StemFn(torch.autograd.Function):
    """Stem forward (with the next BatchNorm's statistics when asked) and weight gradient
    on the MFMA kernels; the input gradient, if one is wanted, from MIOpen."""

    @staticmethod
    def forward(ctx, x, weight, wb, bn_stats=None):
        if bn_stats is not None:
            y, bn_stats.part = stem_hip(x, wb, stats=True)
        else:
            y = stem_hip(x, wb)
        ctx.save_for_backward(x, wb)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _conv_bwd(dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            dw = stem_wgrad_hip(x, dy)
        return dx, dw, None, None


def stem_conv(x: torch.Tensor, conv: nn.Conv2d, wb: torch.Tensor, bn_stats: Optional[BNStats] = None) -> torch.Tensor:
    """``conv(x)`` for the ResNet stem (:func:`stem_fast_ok`) with the bf16 shadow ``wb``."""
    stats["stem"] += 1
    return _StemFn.apply(x, conv.weight, wb, bn_stats)


def kxk_fast_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.numel() > 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros" and isinstance(conv.padding, tuple)
            and wgrad_ok(conv.in_channels, conv.out_channels))


def conv_nhwc(x: torch.Tensor, conv: nn.Conv2d, wb: torch.Tensor, fork: Optional[GradFork] = None,
              bn_stats: Optional[BNStats] = None) -> torch.Tensor:
    """``conv(x)`` with the bf16 weight ``wb`` (the arena shadow), the weight gradient
    going to ``conv.weight`` in fp32 (``fork``: see :class:`GradFork`; ``bn_stats``:
    see :class:`BNStats`, filled only by the 3x3 stride-1 MFMA forward)."""
    pre = getattr(x, "_rla_pre", None)
    if pre is not None:
        # a deferred BatchNorm + ReLU output (ops/bn.py DeferredApply): the 3x3 statistics
        # forward stages the activation itself where that is faster than the apply pass +
        # the regular kernel (timed per shape; the PRE kernel is the run-time-shape
        # instance), else the activation is materialised here
        from .bn import materialize

        if (fork is None and bn_stats is not None and not pre.used and conv3x3_stats_enabled()
                and x.size(1) <= 512 and conv3x3_ok(x, wb, conv.stride, conv.padding)):
            key = (x.size(0) * x.size(2) * x.size(3), x.size(1), wb.size(0), 3, 3, 1, 1)
            tp = _TimingPre(pre)
            be = os.environ.get("RLA_CONV3X3_PRE", "auto")  # pre | apply | auto (timed)
            if be not in ("pre", "apply"):
                be = _pick("fwd_kxk_pre", key, {
                    "pre": lambda: conv3x3_stats_hip(x, wb, tp),
                    "apply": lambda: conv3x3_stats_hip(_applied(x, tp), wb),
                })
            if be == "pre":
                pre.used = True
                stats["fast"] += 1
                stats["pre_applied"] += 1
                return _ConvNHWCFn.apply(x, conv.weight, wb, conv.stride, conv.padding, None, bn_stats, pre)
        x = materialize(x)
    stats["fast"] += 1
    return _ConvNHWCFn.apply(x, conv.weight, wb, conv.stride, conv.padding, fork, bn_stats)
