"""MFMA weight-gradient kernel (csrc/conv_wgrad.hip) against an fp32 PyTorch reference.

The oracle is ``torch.nn.grad.conv2d_weight`` on the fp32 upcasts of the same bf16
``dy`` / ``x``: the kernel multiplies bf16 operands exactly and accumulates in fp32,
so the only difference is the fp32 summation order (relative error ~1e-5 of the
gradient's norm).  Shapes cover every tile configuration of the kernel, row counts
that are not a multiple of the 32/64-row stage, 1 and many row splits, 3x3 with
stride 1 / 2 and padding, and the strided 1x1 of ResNet's downsample branch.
"""
import pytest
import torch

from ray_lightning_accelerators_amd.ops.conv import wgrad_hip, wgrad_ok

pytestmark = pytest.mark.gpu


def _case(n, cin, h, w, cout, k, stride, pad, splits=0, seed=0, algo=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    oh = (h + 2 * pad - k) // stride + 1
    ow = (w + 2 * pad - k) // stride + 1
    x = torch.randn(n, cin, h, w, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(n, cout, oh, ow, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    dy = dy.contiguous(memory_format=torch.channels_last)
    got = wgrad_hip(dy, x, (k, k), (stride, stride), (pad, pad), splits, algo)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, k, k), dy.float(), stride=stride, padding=pad)
    return got, ref


def _check(got, ref, tol=2e-5):
    assert got.dtype == torch.float32 and got.shape == ref.shape
    assert got.is_contiguous(memory_format=torch.channels_last)
    err = (got - ref).norm() / ref.norm()
    assert err < tol, f"normwise error {err:.3e}"
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("cin,cout", [(64, 64), (64, 128), (128, 64), (64, 256), (256, 64), (128, 128), (256, 512)])
def test_wgrad_1x1_tiles(cin, cout):
    got, ref = _case(2, cin, 14, 13, cout, 1, 1, 0)  # M = 364: not a multiple of the stage
    _check(got, ref)


@pytest.mark.parametrize("splits", [1, 3, 0])
def test_wgrad_1x1_splits(splits):
    got, ref = _case(4, 128, 28, 28, 256, 1, 1, 0, splits=splits)
    _check(got, ref)


@pytest.mark.parametrize("k,stride,pad,h", [(3, 1, 1, 14), (3, 2, 1, 15), (1, 2, 0, 14), (3, 1, 0, 9)])
def test_wgrad_kxk(k, stride, pad, h):
    got, ref = _case(2, 64, h, h, 128, k, stride, pad)
    _check(got, ref)


@pytest.mark.parametrize("h,w,n,splits", [(7, 7, 4, 0), (14, 14, 3, 0), (28, 28, 2, 0), (56, 56, 2, 0),
                                          (9, 13, 2, 0), (20, 33, 2, 0), (14, 14, 3, 1), (28, 28, 2, 5)])
def test_wgrad_3x3_halo(h, w, n, splits):
    """3x3 / stride 1 / pad 1: the halo kernel (every output-width class: 16, 32 and
    64-pixel stages; non-square images; one and several splits)."""
    from ray_lightning_accelerators_amd.ops import require

    plan = require().conv_wgrad_plan(n, h, w, 64, h, w, 128, 3, 3, 1, 1, 1, 1, splits)
    assert plan[0] == 1  # halo kernel
    got, ref = _case(n, 64, h, w, 128, 3, 1, 1, splits=splits)
    _check(got, ref)
    gen, _ = _case(n, 64, h, w, 128, 3, 1, 1, splits=splits, algo=1)  # generic tap-GEMM kernel
    _check(gen, ref)


def test_wgrad_resnet_layer1_shape():
    # one of ResNet-50's hottest wgrads at a reduced batch: 56x56, 64 -> 256
    got, ref = _case(8, 64, 56, 56, 256, 1, 1, 0)
    _check(got, ref)
    got, ref = _case(4, 64, 56, 56, 64, 3, 1, 1)
    _check(got, ref)


def test_wgrad_deterministic():
    a, _ = _case(4, 128, 28, 28, 128, 3, 1, 1, seed=3)
    b, _ = _case(4, 128, 28, 28, 128, 3, 1, 1, seed=3)
    assert torch.equal(a, b)


def test_wgrad_rejects_bad_channels():
    assert not wgrad_ok(3, 64) and not wgrad_ok(64, 72)
    x = torch.zeros(1, 32, 4, 4, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.zeros(1, 64, 4, 4, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError):
        wgrad_hip(dy, x, (1, 1), (1, 1), (0, 0))


def test_conv_modules_use_hip_wgrad(monkeypatch):
    """Conv1x1NHWC and ConvBF16 (arena bf16 shadow weights) route their weight
    gradients through the kernel under RLA_CONV_WGRAD=hip; the fp32 gradients match
    the MIOpen backend's (bf16-rounded) ones."""
    from ray_lightning_accelerators_amd.ops import conv as conv_ops
    from ray_lightning_accelerators_amd.ops.conv import Conv1x1NHWC
    from ray_lightning_accelerators_amd.ops.shadow import ConvBF16
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    torch.manual_seed(0)
    m = torch.nn.Sequential(Conv1x1NHWC(64, 128), ConvBF16(128, 64, 3, 1, 1, bias=False)).cuda()
    m = m.to(memory_format=torch.channels_last)
    arena = ParamArena(m)
    arena.enable_bf16_shadow(m)
    x = torch.randn(2, 64, 12, 12, device="cuda").contiguous(memory_format=torch.channels_last)
    calls = {"n": 0}
    real = conv_ops.wgrad_hip

    def counting(*a, **k):
        calls["n"] += 1
        return real(*a, **k)

    monkeypatch.setattr(conv_ops, "wgrad_hip", counting)
    grads = {}
    for mode in ("hip", "miopen"):
        monkeypatch.setenv("RLA_CONV_WGRAD", mode)
        for p in m.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().square().sum().backward()
        grads[mode] = [p.grad.detach().float().clone() for p in m.parameters()]
    assert calls["n"] == 2  # one per layer, hip mode only
    for got, ref in zip(grads["hip"], grads["miopen"]):
        err = (got - ref).norm() / ref.norm()
        assert err < 1e-2, err
