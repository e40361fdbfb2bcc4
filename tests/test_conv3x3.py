"""3x3 / stride 1 / pad 1 NHWC convolution on MFMA (csrc/conv3x3.hip): forward and
input gradient against an fp32 PyTorch reference of the same bf16 operands."""
import pytest
import torch
import torch.nn.functional as F

gpu = pytest.mark.gpu

# (N, H, W, Cin, Cout): ResNet-50's stride-1 conv2 shapes at small batch, plus tiles
# that cross image boundaries (H*W not a multiple of 256, tiny images) and a tail
SHAPES = [
    (2, 56, 56, 64, 64),
    (2, 28, 28, 128, 128),
    (3, 14, 14, 256, 256),
    (5, 7, 7, 512, 512),
    (3, 5, 9, 16, 64),
    (1, 3, 3, 32, 128),
    (7, 11, 13, 48, 64),
]


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(params=["256", "512"])
def tile_px(request, monkeypatch):
    """Both workgroup tile sizes (the host picks 512 pixels only for large layers)."""
    monkeypatch.setenv("RLA_CONV3X3_TM", request.param)
    return int(request.param)


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_forward_matches_fp32(shape, tile_px):
    from ray_lightning_accelerators_amd import ops
    from ray_lightning_accelerators_amd.ops.conv import conv3x3_hip

    n, h, w, cin, cout = shape
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = (torch.randn(cout, cin, 3, 3, device=dev) / (3 * cin ** 0.5)).to(torch.bfloat16)
    wb = wb.contiguous(memory_format=torch.channels_last)
    assert ops.require().conv3x3_supported(n, h, w, cin, cout)
    y = conv3x3_hip(x, wb)
    ref = F.conv2d(x.float(), wb.float(), padding=1)
    assert y.shape == ref.shape and y.dtype == torch.bfloat16
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 8e-3, _rel(y, ref)  # bf16 output rounding (2^-9 relative)
    assert float((y.float() - ref).abs().max()) < 0.05 * float(ref.abs().max())


@gpu
@pytest.mark.parametrize("shape", SHAPES[:4] + SHAPES[-1:])
def test_conv3x3_dgrad_matches_fp32(shape, tile_px):
    from ray_lightning_accelerators_amd.ops.conv import conv3x3_dgrad_hip

    n, h, w, cin, cout = shape
    if cout % 64 or cin % 64:  # the dgrad swaps the channel roles: Cin becomes the tile side
        pytest.skip("dgrad needs Cin % 64 == 0")
    torch.manual_seed(1)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, cin, h, w, device=dev, requires_grad=True)
    wb = (torch.randn(cout, cin, 3, 3, device=dev) / (3 * cin ** 0.5)).to(torch.bfloat16)
    wb = wb.contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    F.conv2d(x, wb.float(), padding=1).backward(dy.float())
    dx = conv3x3_dgrad_hip(dy, wb)
    assert dx.shape == x.shape
    assert _rel(dx, x.grad) < 8e-3, _rel(dx, x.grad)


@gpu
def test_conv_bf16_layer_routes_through_kernel(monkeypatch):
    """ConvBF16 with an arena shadow: RLA_CONV3X3 auto-times the kernel against
    MIOpen per shape; forced to the kernel, the layer's output and input gradient
    match MIOpen's (both bf16 convolutions of the same operands)."""
    from ray_lightning_accelerators_amd.ops import conv as C
    from ray_lightning_accelerators_amd.ops.shadow import ConvBF16
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = torch.nn.ModuleList([ConvBF16(64, 64, 3, 1, 1, bias=False)]).to(dev).to(memory_format=torch.channels_last)
    arena = ParamArena(m)
    arena.enable_bf16_shadow(m)
    x0 = torch.randn(4, 64, 20, 20, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    calls = {"fwd": 0, "dgrad": 0}
    real_f, real_d = C.conv3x3_hip, C.conv3x3_dgrad_hip

    def fwd(*a, **k):
        calls["fwd"] += 1
        return real_f(*a, **k)

    def dgrad(*a, **k):
        calls["dgrad"] += 1
        return real_d(*a, **k)

    monkeypatch.setattr(C, "conv3x3_hip", fwd)
    monkeypatch.setattr(C, "conv3x3_dgrad_hip", dgrad)
    outs = {}
    for mode in ("hip", "miopen"):
        monkeypatch.setenv("RLA_CONV1X1", mode)  # _pick honours a pinned backend name
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m[0](x)
        y.float().square().sum().backward()
        outs[mode] = (y.detach().float(), x.grad.float())
        if mode == "hip":
            assert calls["fwd"] >= 1 and calls["dgrad"] >= 1
    assert _rel(outs["hip"][0], outs["miopen"][0]) < 1e-2
    assert _rel(outs["hip"][1], outs["miopen"][1]) < 2e-2


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_stats_epilogue(shape, tile_px):
    """The forward's BatchNorm partial sums (ST epilogue): same y as the plain kernel,
    and the rows sum to the per-channel sum / sum of squares of the bf16 output."""
    from ray_lightning_accelerators_amd.ops.conv import conv3x3_hip, conv3x3_stats_hip

    n, h, w, cin, cout = shape
    torch.manual_seed(2)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = (torch.randn(cout, cin, 3, 3, device=dev) / (3 * cin ** 0.5)).to(torch.bfloat16)
    wb = wb.contiguous(memory_format=torch.channels_last)
    y, part = conv3x3_stats_hip(x, wb)
    assert torch.equal(y, conv3x3_hip(x, wb))
    assert part.dim() == 3 and part.size(1) == 2 and part.size(2) == cout and part.dtype == torch.float32
    yf = y.double().permute(0, 2, 3, 1).reshape(-1, cout)
    s, q = part.double().sum(0)
    torch.testing.assert_close(s, yf.sum(0), rtol=1e-4, atol=1e-3 * yf.abs().sum(0).max().item() / yf.size(0) ** 0.5)
    torch.testing.assert_close(q, yf.square().sum(0), rtol=1e-4, atol=1e-3)


@gpu
def test_resnet_block_bn2_uses_conv3x3_stats(monkeypatch):
    """A bottleneck's conv2 hands bn2 its epilogue statistics (RLA_CONV3X3_STATS auto,
    the kernel pinned): the block's output and gradients match the path where bn2 runs
    its own partial pass."""
    from ray_lightning_accelerators_amd.models.resnet import Bottleneck
    from ray_lightning_accelerators_amd.ops import conv as C
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    dev = torch.device("cuda", 0)
    calls = {"st": 0}
    real = C.conv3x3_stats_hip

    def st(*a, **k):
        calls["st"] += 1
        return real(*a, **k)

    monkeypatch.setattr(C, "conv3x3_stats_hip", st)
    monkeypatch.setenv("RLA_CONV1X1", "hip_st")  # pins the stats kernel in _pick (other ops: auto)
    outs = {}
    for mode in ("auto", "off"):
        monkeypatch.setenv("RLA_CONV3X3_STATS", mode)
        torch.manual_seed(0)
        blk = Bottleneck(256, 64, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
        arena = ParamArena(blk)
        arena.enable_bf16_shadow(blk)
        torch.manual_seed(1)
        x = torch.randn(4, 256, 14, 14, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
        y.float().square().mean().backward()
        outs[mode] = (y.detach().float(), x.grad.float(), blk.conv2.weight.grad.clone(), blk.bn2.running_var.clone())
    assert calls["st"] >= 1
    for a, b in zip(outs["auto"], outs["off"]):
        assert _rel(a, b.float()) < 2e-2, _rel(a, b.float())


STEM_SHAPES = [(2, 224, 224), (3, 32, 32), (2, 30, 46), (1, 17, 20)]


@gpu
@pytest.mark.parametrize("shape", STEM_SHAPES)
def test_stem_forward_and_stats_match_fp32(shape):
    """ResNet stem on the MFMA kernel (csrc/stem.hip): 7x7 / stride 2 / pad 3, 3 -> 64,
    against an fp32 conv of the same bf16 operands; the statistics rows sum to the
    per-channel sums of the bf16 output."""
    from ray_lightning_accelerators_amd.ops.conv import stem_hip

    n, h, w = shape
    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, 3, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = (torch.randn(64, 3, 7, 7, device=dev) / 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = stem_hip(x, wb)
    ref = F.conv2d(x.float(), wb.float(), stride=2, padding=3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 8e-3, _rel(y, ref)
    y2, part = stem_hip(x, wb, stats=True)
    assert torch.equal(y, y2)
    yf = y.double().permute(0, 2, 3, 1).reshape(-1, 64)
    s, q = part.double().sum(0)
    torch.testing.assert_close(s, yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(q, yf.square().sum(0), rtol=1e-4, atol=1e-2)


@gpu
def test_resnet_stem_routes_through_kernel(monkeypatch):
    """The fused ResNet's stem runs the MFMA kernel with bn1's statistics; output and
    the stem weight's gradient match RLA_STEM=off (MIOpen forward + bn1's own pass)."""
    from ray_lightning_accelerators_amd.models.resnet import resnet50
    from ray_lightning_accelerators_amd.ops import conv as C
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    dev = torch.device("cuda", 0)
    outs = {}
    for mode in ("auto", "off"):
        monkeypatch.setenv("RLA_STEM", mode)
        C._stem_shape_ok.cache_clear()
        torch.manual_seed(0)
        m = resnet50(num_classes=10, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
        arena = ParamArena(m)
        arena.enable_bf16_shadow(m)
        torch.manual_seed(1)
        x = torch.randn(2, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
        before = C.stats["stem"]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            st = C.BNStats()
            y = m.bn1(m.conv1(x, bn_stats=st), bn_stats=st)
        y.float().square().mean().backward()
        used = C.stats["stem"] - before
        assert (used >= 1) == (mode == "auto"), (mode, used)
        outs[mode] = (y.detach().float(), m.conv1.weight.grad.clone(), m.bn1.running_var.clone())
    for a, b in zip(outs["auto"], outs["off"]):
        assert _rel(a, b.float()) < 2e-2, _rel(a, b.float())


@gpu
def test_bn_relu_folded_into_maxpool_matches_unfused():
    """bn1 + ReLU inside the max pool's pass (ops/bn.py ``pool``): pooled output,
    running statistics and every gradient equal the unfused bn -> pool pair."""
    from ray_lightning_accelerators_amd.ops.bn import BatchNormAct2d
    from ray_lightning_accelerators_amd.ops.pool import MaxPool2dNHWC

    dev = torch.device("cuda", 0)
    torch.manual_seed(4)
    x0 = torch.randn(3, 64, 22, 18, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g0 = torch.randn(3, 64, 11, 9, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for fold in (True, False):
        torch.manual_seed(5)
        bn = BatchNormAct2d(64).to(dev)
        with torch.no_grad():
            bn.weight.uniform_(-1, 1)  # negative scales too: the affine map is not monotone
            bn.bias.uniform_(-0.5, 0.5)
        pool = MaxPool2dNHWC(3, 2, 1)
        x = x0.clone().requires_grad_(True)
        y = bn(x, pool=pool) if fold else pool(bn(x))
        y.backward(g0)
        outs.append((y.detach(), x.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var,
                     bn.num_batches_tracked))
    for a, b in zip(*outs):
        assert torch.equal(a, b), (a - b).abs().max() if a.is_floating_point() else (a, b)


@gpu
@pytest.mark.parametrize("shape", STEM_SHAPES)
def test_stem_wgrad_matches_fp32(shape):
    """Stem weight gradient on the MFMA kernel against fp32 autograd of the same bf16 operands."""
    from ray_lightning_accelerators_amd.ops.conv import stem_wgrad_hip

    n, h, w = shape
    torch.manual_seed(6)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, 3, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    dy = torch.randn(n, 64, oh, ow, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w32 = torch.zeros(64, 3, 7, 7, device=dev, requires_grad=True)
    F.conv2d(x.float(), w32, stride=2, padding=3).backward(dy.float())
    dw = stem_wgrad_hip(x, dy)
    assert dw.shape == (64, 3, 7, 7) and dw.dtype == torch.float32
    assert dw.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dw, w32.grad) < 1e-4, _rel(dw, w32.grad)


def _stats4(c, dev, seed):
    """bn_finalize's [4, C] layout with random scale / shift (both signs: the ReLU clips
    either way)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    st = torch.randn(4, c, generator=g)
    st[1] = st[1].abs() + 0.5
    return st.to(dev).contiguous()


def _apply_nhwc(x, st):
    from ray_lightning_accelerators_amd import ops

    y = torch.empty_like(x)
    ops.require().bn_apply(x, st[2].contiguous(), st[3].contiguous(), None, True, y)
    return y


@gpu
@pytest.mark.parametrize("shape", SHAPES[:4] + SHAPES[-1:])
def test_conv3x3_pre_matches_materialized(shape, tile_px):
    """A deferred BatchNorm + ReLU staged by the 3x3 statistics forward (csrc/conv3x3.hip
    PRE): y and the partial sums bitwise those of the kernel on the materialised
    activation, the zero padding untouched (fp32 reference of conv(relu(x*s+b))), and
    num_batches_tracked incremented once."""
    from ray_lightning_accelerators_amd import ops

    n, h, w, cin, cout = shape
    torch.manual_seed(9)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, h, w, cin, device=dev).to(torch.bfloat16)
    wt = (torch.randn(cout, 3, 3, cin, device=dev) / (9 * cin) ** 0.5).to(torch.bfloat16)
    st = _stats4(cin, dev, 10)
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    y1, p1 = ops.require().conv3x3_stats(x, wt, n, h, w, cin, cout, st, nbt)
    a = _apply_nhwc(x, st)
    y0, p0 = ops.require().conv3x3_stats(a, wt, n, h, w, cin, cout)
    assert int(nbt) == 1
    ref = F.conv2d(a.float().permute(0, 3, 1, 2), wt.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(y1, ref) < 8e-3, _rel(y1, ref)
    # the PRE kernel is the run-time-shape instance; the materialised run may take a
    # compile-time-shape one: the same MFMA order, so bitwise equal
    assert torch.equal(y1, y0), float((y1.float() - y0.float()).abs().max())
    assert torch.equal(p1, p0)


@gpu
@pytest.mark.parametrize("shape", [(2, 28, 28, 64, 64), (3, 14, 14, 128, 128), (2, 7, 7, 512, 512)])
@pytest.mark.parametrize("algo", [0, 1])
def test_wgrad3x3_pre_matches_materialized(shape, algo):
    """The 3x3 weight gradient staging relu(x * scale + shift) itself (halo kernel,
    algo 0; generic tap kernel, algo 1; csrc/conv_wgrad.hip PRE) == the same kernel on
    the materialised activation, bitwise; padding taps stay zero."""
    from ray_lightning_accelerators_amd import ops

    n, h, w, cin, cout = shape
    torch.manual_seed(11)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, h, w, cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(n, h, w, cout, device=dev).to(torch.bfloat16)
    st = _stats4(cin, dev, 12)
    geo = (n, h, w, cin, h, w, cout, 3, 3, 1, 1, 1, 1)
    g1 = ops.require().conv_wgrad(dy, x, *geo, 0, algo, st)
    g0 = ops.require().conv_wgrad(dy, _apply_nhwc(x, st), *geo, 0, algo)
    assert torch.equal(g1, g0)


@gpu
def test_resnet_block_bn1_deferred_into_conv2(monkeypatch):
    """A training identity Bottleneck with a parameter arena (conv2 on the 3x3 kernel):
    bn1 + ReLU deferred into conv2 (and bn2 into conv3) == the block with both apply
    passes -- output, input gradient, every parameter gradient and bn1's running
    statistics bitwise."""
    from ray_lightning_accelerators_amd.models.resnet import Bottleneck
    from ray_lightning_accelerators_amd.ops import bn as B
    from ray_lightning_accelerators_amd.ops import conv as C
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    monkeypatch.setenv("RLA_CONV1X1", "hip")
    monkeypatch.setenv("RLA_CONV_WGRAD", "hip")
    monkeypatch.setenv("RLA_CONV3X3_PRE", "pre")
    dev = torch.device("cuda", 0)
    torch.manual_seed(13)
    blk = Bottleneck(256, 64, 1, None, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    arena = ParamArena(blk)
    arena.enable_bf16_shadow(blk)
    x0 = torch.randn(2, 256, 28, 28, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    outs = []
    for defer in ("0", "1"):
        monkeypatch.setenv("RLA_BN_DEFER", defer)
        blk.load_state_dict(state)
        blk.zero_grad(set_to_none=True)
        n0, a0 = B.fold_stats["deferred"], C.stats["pre_applied"]
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
        y.float().square().mean().backward()
        if defer == "1":
            assert B.fold_stats["deferred"] - n0 == 2 and C.stats["pre_applied"] - a0 == 2
        outs.append((y.detach().float(), x.grad.float(), [p.grad.detach().clone() for p in blk.parameters()],
                     blk.bn1.running_mean.clone(), blk.bn1.running_var.clone(), int(blk.bn1.num_batches_tracked)))
    (y0, g0, p0, m0, v0, n0), (y1, g1, p1, m1, v1, n1) = outs
    assert torch.equal(y0, y1)
    assert torch.equal(g0, g1)
    for nm, a, b in zip([n for n, _ in blk.named_parameters()], p0, p1):
        assert torch.equal(a, b), nm
    assert torch.equal(m0, m1) and torch.equal(v0, v1) and n0 == n1 == 1
