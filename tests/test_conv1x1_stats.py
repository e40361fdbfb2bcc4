"""1x1 convolution forward with the next BatchNorm's statistics in its epilogue
(csrc/conv1x1.hip): the output against an fp32 PyTorch reference of the same bf16
operands, the partial sums against fp64 sums of the kernel's own bf16 output, and
the BatchNorm that consumes them against the same layer running its own partial
pass (outputs, running statistics, num_batches_tracked)."""
import pytest
import torch
import torch.nn.functional as F

gpu = pytest.mark.gpu

# (M, K, N): ResNet-50 1x1 shapes at small batch, a pixel tail (M % 128 != 0), a
# column count that is not a multiple of 128 (one 32-channel block per wave), K = 32;
# together they reach every launch variant (resident weights at 2 or 1 workgroups
# per CU, streamed weights, 32- and 64-channel wave columns)
SHAPES = [
    (2 * 56 * 56, 64, 256),
    (2 * 56 * 56, 256, 64),
    (3 * 28 * 28, 512, 128),
    (5 * 7 * 7, 512, 2048),
    (4 * 14 * 14, 1024, 256),
    (3 * 28 * 28, 128, 512),
    (1000, 64, 192),
    (300, 1024, 192),
    (77, 32, 64),
]


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm().clamp_min(1e-30))


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_conv1x1_stats_matches_fp32(shape):
    from ray_lightning_accelerators_amd import ops

    m, k, n = shape
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    wb = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    y, part = ops.require().conv1x1_stats(x, wb)
    ref = x.float() @ wb.float().t()
    assert y.shape == (m, n) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 8e-3, _rel(y, ref)
    assert part.dim() == 3 and part.size(1) == 2 and part.size(2) == n and part.size(0) % 8 == 0
    yd = y.double()
    s = part.double().sum(0)
    # the sums are of the ROUNDED outputs the kernel stored (what bn_partial would read)
    assert torch.allclose(s[0], yd.sum(0), rtol=1e-4, atol=1e-3 * m ** 0.5)
    assert torch.allclose(s[1], (yd * yd).sum(0), rtol=1e-4, atol=1e-3)


@gpu
def test_conv1x1_stats_deterministic():
    from ray_lightning_accelerators_amd import ops

    torch.manual_seed(1)
    dev = torch.device("cuda", 0)
    x = torch.randn(3 * 56 * 56, 64, device=dev).to(torch.bfloat16)
    wb = torch.randn(256, 64, device=dev).to(torch.bfloat16)
    y0, p0 = ops.require().conv1x1_stats(x, wb)
    y1, p1 = ops.require().conv1x1_stats(x, wb)
    assert torch.equal(y0, y1) and torch.equal(p0, p1)


@gpu
@pytest.mark.parametrize("residual", [False, True])
def test_bn_consumes_conv_epilogue_stats(residual, monkeypatch):
    """BatchNormAct2d fed the conv's partial sums == the same layer summing the same
    conv output itself (both runs take the kernel's y; one drops its partials)."""
    from ray_lightning_accelerators_amd.ops.bn import BatchNormAct2d
    from ray_lightning_accelerators_amd.ops.conv import BNStats, Conv1x1NHWC

    torch.manual_seed(2)
    dev = torch.device("cuda", 0)
    conv = Conv1x1NHWC(64, 128).to(dev)
    x0 = torch.randn(4, 64, 20, 20, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn(4, 128, 20, 20, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    monkeypatch.setenv("RLA_CONV1X1", "hip")
    outs = []
    for use in (False, True):
        bn = BatchNormAct2d(128).to(dev)
        bn.momentum = None  # cumulative average: the finalize reads num_batches_tracked
        x = x0.clone().requires_grad_(True)
        for _ in range(2):
            st = BNStats()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = conv(x, bn_stats=st)
                assert st.part is not None
                if not use:
                    st.part = None  # the layer sums y itself
                z = bn(y, res if residual else None, bn_stats=st)
        z.float().square().sum().backward()
        outs.append((z.detach().float(), x.grad.float(), bn.running_mean.clone(), bn.running_var.clone(),
                     int(bn.num_batches_tracked)))
    (z0, g0, m0, v0, n0), (z1, g1, m1, v1, n1) = outs
    assert n0 == n1 == 2
    assert _rel(z1, z0) < 1e-5
    assert _rel(g1, g0) < 1e-4
    assert torch.allclose(m1, m0, rtol=1e-5, atol=1e-6) and torch.allclose(v1, v0, rtol=1e-5, atol=1e-6)


@gpu
def test_resnet_bottleneck_routes_stats(monkeypatch):
    """A training Bottleneck pinned to the kernel computes its 1x1 layers' BN
    statistics in the conv epilogue (conv1 / conv3 / stride-1 downsample)."""
    from ray_lightning_accelerators_amd.models.resnet import Bottleneck
    from ray_lightning_accelerators_amd.ops import conv as C
    from torch import nn

    monkeypatch.setenv("RLA_CONV1X1", "hip")
    calls = {"n": 0}
    real = C.conv1x1_stats_hip

    def spy(*a, **k):
        calls["n"] += 1
        return real(*a, **k)

    monkeypatch.setattr(C, "conv1x1_stats_hip", spy)
    from ray_lightning_accelerators_amd.ops.bn import BatchNormAct2d

    dev = torch.device("cuda", 0)
    down = nn.Sequential(C.Conv1x1NHWC(64, 256), BatchNormAct2d(256, act=None))
    blk = Bottleneck(64, 64, 1, down, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(2, 64, 16, 16, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
    y.float().sum().backward()
    assert calls["n"] == 3
    assert int(blk.bn1.num_batches_tracked) == int(blk.bn3.num_batches_tracked) == 1
    assert int(blk.bn2.num_batches_tracked) == 1  # deferred apply: conv3's kernel counted it
    assert int(down[1].num_batches_tracked) == 1
    assert torch.isfinite(x.grad.float()).all()


@gpu
@pytest.mark.parametrize("shape", [(2 * 56 * 56, 64, 256), (3 * 28 * 28, 128, 512), (1000, 32, 192), (77, 64, 64)])
def test_conv1x1_bn_bwd_matches_reference(shape):
    """Input gradient + previous BatchNorm backward partial in one kernel: d against
    bf16((bf16(dy1 . W) + dy2) * (yb > 0)) from an fp32 GEMM (one bf16 ulp where the
    GEMM's fp32 sums round differently), the partial sums against fp64 sums of the
    kernel's own d."""
    from ray_lightning_accelerators_amd import ops

    m, k, n = shape
    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    dy1 = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(k, n, device=dev) / k ** 0.5).to(torch.bfloat16)  # conv weight [Cout = k, Cin = n]
    dy2 = torch.randn(m, n, device=dev).to(torch.bfloat16)
    yb = torch.randn(m, n, device=dev).to(torch.bfloat16).clamp_min(0)  # a ReLU output (zeros included)
    xb = torch.randn(m, n, device=dev).to(torch.bfloat16)
    d, part = ops.require().conv1x1_bn_bwd(dy1, w.t().contiguous(), dy2, yb, xb)
    da = (dy1.float() @ w.float()).to(torch.bfloat16)
    ref = ((da.float() + dy2.float()) * (yb.float() > 0)).to(torch.bfloat16)
    assert d.shape == (m, n) and d.dtype == torch.bfloat16
    assert _rel(d, ref.float()) < 8e-3, _rel(d, ref.float())
    assert torch.equal(d == 0, ref == 0) or bool(((d == 0) != (ref == 0)).float().mean() < 1e-3)
    s = part.double().sum(0)
    dd = d.double()
    assert torch.allclose(s[0], dd.sum(0), rtol=1e-4, atol=1e-3 * m ** 0.5)
    assert torch.allclose(s[1], (dd * xb.double()).sum(0), rtol=1e-4, atol=1e-3 * m ** 0.5)


@gpu
def test_fused_bn_dgrad_resnet_layer_matches(monkeypatch):
    """ResNet-50 layer1 (three bottlenecks, two identity shortcuts) with the fused conv1
    input gradient + bn3 backward partial: the same loss and gradients as the unfused
    step (the GEMM rounds differently: bf16-level tolerances)."""
    from ray_lightning_accelerators_amd.models.resnet import resnet50
    from ray_lightning_accelerators_amd.ops import conv as C

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    full = resnet50(num_classes=10, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    layer = full.layer1
    x0 = torch.randn(4, 64, 32, 32, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("RLA_FUSE_BN_DGRAD", fuse)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        n0 = C.stats["bn_dgrad_fused"]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = layer(x)
        y.float().square().mean().backward()
        assert C.stats["bn_dgrad_fused"] - n0 == (2 if fuse == "1" else 0)  # the two identity blocks' conv1
        outs.append((y.detach().float(), x.grad.float(),
                     [p.grad.detach().float().clone() for p in layer.parameters()]))
    (y0, g0, p0), (y1, g1, p1) = outs
    assert torch.equal(y0, y1)
    assert _rel(g1, g0) < 2e-2, _rel(g1, g0)
    for a, b in zip(p1, p0):
        assert _rel(a, b) < 3e-2, _rel(a, b)



@gpu
def test_fused_bn_dgrad_guard_with_extra_consumer(monkeypatch):
    """an extra autograd consumer of an identity block's output (a feature
    tap) makes autograd hand bn3 the SUM of the conv's d and the tap's gradient; the
    conv's fused partial sums are of d alone, so bn3 must notice and run its own
    partial pass -- gradients then match the unfused step."""
    from ray_lightning_accelerators_amd.models.resnet import resnet50
    from ray_lightning_accelerators_amd.ops import bn as B

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    layer = resnet50(num_classes=10, fused_bn=True).to(dev).to(memory_format=torch.channels_last).layer1
    x0 = torch.randn(4, 64, 32, 32, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("RLA_FUSE_BN_DGRAD", fuse)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        r0 = B.fold_stats["fused_rejected"]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            h = layer[0](x)           # identity-block input: read by layer[1].conv1 ...
            tap = h.float().mean()    # ... and by a feature tap
            y = layer[2](layer[1](h))
        (y.float().square().mean() + 10.0 * tap).backward()
        if fuse == "1":
            assert B.fold_stats["fused_rejected"] - r0 >= 1
        outs.append((x.grad.float(), [p.grad.detach().float().clone() for p in layer.parameters()]))
    (g0, p0), (g1, p1) = outs
    assert _rel(g1, g0) < 2e-2, _rel(g1, g0)
    for a, b in zip(p1, p0):
        assert _rel(a, b) < 3e-2, _rel(a, b)


def _stats4(k, dev, seed):
    """bn_finalize's [4, K] layout (mean, invstd, scale, shift) with random scale /
    shift -- negative scales and shifts included, so the ReLU clips both ways."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    st = torch.randn(4, k, generator=g)
    st[1] = st[1].abs() + 0.5
    return st.to(dev).contiguous()


def _apply(x, st):
    """The materialised activation from the production apply kernel (bf16(relu(x * scale
    + shift)))."""
    from ray_lightning_accelerators_amd import ops

    y = torch.empty_like(x)
    ops.require().bn_apply(x, st[2].contiguous(), st[3].contiguous(), None, True, y)
    return y


@gpu
@pytest.mark.parametrize("shape", [(2 * 56 * 56, 64, 256), (3 * 28 * 28, 128, 512), (1000, 64, 192), (77, 32, 64),
                                   (300, 256, 128)])
def test_conv1x1_pre_matches_materialized(shape):
    """A deferred BatchNorm + ReLU applied inside the 1x1 forward (csrc/conv1x1.hip PRE)
    == the same kernel on the activation materialised by the apply kernel: y and the
    partial sums bitwise, and num_batches_tracked incremented once."""
    from ray_lightning_accelerators_amd import ops

    m, k, n = shape
    torch.manual_seed(4)
    dev = torch.device("cuda", 0)
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    wb = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    st = _stats4(k, dev, 5)
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    y1, p1 = ops.require().conv1x1_stats(x, wb, st, nbt)
    y0, p0 = ops.require().conv1x1_stats(_apply(x, st), wb)
    assert torch.equal(y1, y0)
    assert torch.equal(p1, p0)
    assert int(nbt) == 1
    a = torch.relu(x.float() * st[2] + st[3]).to(torch.bfloat16).float()
    assert _rel(y1, a @ wb.float().t()) < 8e-3


@gpu
@pytest.mark.parametrize("shape", [(2 * 28 * 28, 64, 256), (3 * 14 * 14, 128, 512), (500, 64, 64)])
def test_wgrad_pre_matches_materialized(shape):
    """The weight gradient staging relu(x * scale + shift) itself (csrc/conv_wgrad.hip
    PRE) == the kernel on the materialised activation, bitwise (fp32 [Cout, Cin])."""
    from ray_lightning_accelerators_amd import ops

    m, cin, cout = shape
    torch.manual_seed(6)
    dev = torch.device("cuda", 0)
    x = torch.randn(m, cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(m, cout, device=dev).to(torch.bfloat16)
    st = _stats4(cin, dev, 7)
    geo = (1, m, 1, cin, m, 1, cout, 1, 1, 1, 1, 0, 0)
    g1 = ops.require().conv_wgrad(dy, x, *geo, 0, 0, st)
    g0 = ops.require().conv_wgrad(dy, _apply(x, st), *geo, 0, 0)
    assert torch.equal(g1, g0)
    ref = dy.float().t() @ torch.relu(x.float() * st[2] + st[3]).to(torch.bfloat16).float()
    assert _rel(g1.view(cout, cin), ref) < 1e-4


@gpu
@pytest.mark.parametrize("down", [False, True])
def test_bottleneck_deferred_bn2_matches_applied(down, monkeypatch):
    """A training Bottleneck with bn2's apply deferred into conv3 (RLA_BN_DEFER=1, the
    default) == the same block with the apply pass (RLA_BN_DEFER=0): output, input
    gradient, every parameter gradient and bn2's running statistics bitwise."""
    from ray_lightning_accelerators_amd.models.resnet import Bottleneck
    from ray_lightning_accelerators_amd.ops import bn as B
    from ray_lightning_accelerators_amd.ops import conv as C
    from ray_lightning_accelerators_amd.ops.bn import BatchNormAct2d
    from torch import nn

    monkeypatch.setenv("RLA_CONV1X1", "hip")  # one forward backend for both runs
    monkeypatch.setenv("RLA_CONV_WGRAD", "hip")  # one weight-gradient backend for both runs
    dev = torch.device("cuda", 0)
    torch.manual_seed(8)
    cin = 64 if down else 256
    ds = nn.Sequential(C.Conv1x1NHWC(64, 256), BatchNormAct2d(256, act=None)) if down else None
    blk = Bottleneck(cin, 64, 1, ds, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    x0 = torch.randn(2, cin, 20, 20, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    outs = []
    for defer in ("0", "1"):
        monkeypatch.setenv("RLA_BN_DEFER", defer)
        blk.load_state_dict(state)
        blk.zero_grad(set_to_none=True)
        n0, a0, m0_ = B.fold_stats["deferred"], C.stats["pre_applied"], B.fold_stats["materialized"]
        x = x0.clone().requires_grad_(True)
        for _ in range(2):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = blk(x)
        y.float().square().mean().backward()
        if defer == "1":
            # bn1 and bn2 defer; conv3 applies bn2 itself, conv2 (a plain autocast conv:
            # no arena here) gets bn1's activation materialised
            assert B.fold_stats["deferred"] - n0 == 4 and C.stats["pre_applied"] - a0 == 2
            assert B.fold_stats["materialized"] - m0_ == 2
        outs.append((y.detach().float(), x.grad.float(), [p.grad.detach().clone() for p in blk.parameters()],
                     blk.bn2.running_mean.clone(), blk.bn2.running_var.clone(), int(blk.bn2.num_batches_tracked)))
    (y0, g0, p0, m0, v0, n0), (y1, g1, p1, m1, v1, n1) = outs
    assert torch.equal(y0, y1)
    assert torch.equal(g0, g1)
    for nm, a, b in zip([n for n, _ in blk.named_parameters()], p0, p1):
        if nm == "conv2.weight":
            # without a parameter arena conv2 is a plain autocast nn.Conv2d whose MIOpen
            # weight gradient differs run to run at the 1e-7 level (split-K atomics):
            # not bitwise even between two runs of the same mode
            assert _rel(a, b.float()) < 1e-4, (nm, _rel(a, b.float()))
        else:
            assert torch.equal(a, b), nm
    assert torch.equal(m0, m1) and torch.equal(v0, v1) and n0 == n1 == 2
