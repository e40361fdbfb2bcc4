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
