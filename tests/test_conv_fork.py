"""GradFork: a bottleneck's conv1 and downsample conv accumulate their input
gradients into ONE tensor (ops/conv.py) -- the gradient equals autograd's sum."""
import pytest
import torch

from ray_lightning_accelerators_amd.ops import conv as C

gpu = pytest.mark.gpu


def test_fork_dx_order_independent_cpu():
    a, b = torch.randn(2, 8, 4, 4), torch.randn(2, 8, 4, 4)
    for first, second in ((a, b), (b, a)):
        f = C.GradFork()
        f.users = 2
        assert C._fork_dx(f, lambda: first.clone(), None) is None
        out = C._fork_dx(f, lambda: second.clone(), None)
        assert torch.allclose(out, a + b) and f.dx is None
    f = C.GradFork()
    f.users = 1  # the other consumer is on a stock path: no parking
    assert torch.equal(C._fork_dx(f, lambda: a, None), a)


@gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_forked_convs_match_autograd_sum(stride):
    """conv1 (1x1, stride 1, GEMM / MIOpen) and the downsample conv (1x1, stride s)
    on the same input: x.grad with the fork equals the plain two-branch autograd sum
    (fp32 reference of the same bf16 ops), for both backward orders."""
    from ray_lightning_accelerators_amd.ops.shadow import ConvBF16
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    cin, width, cout = 64, 64, 256
    c1 = C.Conv1x1NHWC(cin, width).to(dev)
    ds = (C.Conv1x1NHWC(cin, cout) if stride == 1 else ConvBF16(cin, cout, 1, stride, bias=False)).to(dev)
    pair = torch.nn.ModuleList([c1, ds]).to(memory_format=torch.channels_last)
    # ConvBF16 takes its native (fork-aware) path only with an arena bf16 shadow
    arena = ParamArena(pair)
    arena.enable_bf16_shadow(pair)
    x0 = torch.randn(4, cin, 16, 16, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(use_fork, swap):
        x = x0.clone().requires_grad_(True)
        fork = C.GradFork() if use_fork else None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if swap:
                a = c1(x, fork=fork)
                b = ds(x, fork=fork)
            else:
                b = ds(x, fork=fork)
                a = c1(x, fork=fork)
        g = torch.Generator(device=dev).manual_seed(1)
        ga = torch.randn(a.shape, device=dev, generator=g)
        gb = torch.randn(b.shape, device=dev, generator=g)
        (a.float() * ga.float()).sum().add_((b.float() * gb.float()).sum()).backward()
        if use_fork:
            assert fork.users == 2 and fork.dx is None
        return x.grad.float(), c1.weight.grad.clone(), ds.weight.grad.clone()

    for swap in (False, True):
        c1.weight.grad = ds.weight.grad = None
        ref = run(False, swap)
        c1.weight.grad = ds.weight.grad = None
        got = run(True, swap)
        err = (got[0] - ref[0]).norm() / ref[0].norm()
        assert err < 2e-2, err  # bf16 dgrad outputs, different rounding points
        assert torch.allclose(got[1], ref[1]) and torch.allclose(got[2], ref[2])


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,h,w,s", [(2, 256, 56, 56, 2), (3, 64, 15, 9, 2), (1, 32, 7, 7, 3), (2, 16, 8, 8, 1)])
def test_strided_add_matches_aten_bitwise(n, c, h, w, s):
    """The fork's strided add (csrc/pool.hip strided_add_kernel) against ATen's bf16
    add_ on the strided view: fp32 add and one rounding in both, so bitwise equal."""
    import torch

    from ray_lightning_accelerators_amd.ops import require

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(n * 100 + c)
    d = torch.randn(n, c, h, w, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
    g2 = torch.randn(n * oh * ow, c, generator=g).to(dev, torch.bfloat16)
    ref = d.clone()
    ref[:, :, ::s, ::s].add_(g2.view(n, oh, ow, c).permute(0, 3, 1, 2))
    require().strided_add_(d, g2, s)
    torch.cuda.synchronize()
    assert torch.equal(d.view(torch.int16), ref.view(torch.int16))
