"""Weight gradients on a side stream (ops/conv.py, RLA_WGRAD_STREAM=1): a ResNet-50
training step through the fused ops produces bitwise the same arena gradients as
with every weight gradient on the backward's own stream -- eager, and replayed from
a captured graph."""
import pytest
import torch
import torch.nn.functional as F

gpu = pytest.mark.gpu


def _model(dev):
    from ray_lightning_accelerators_amd.models.resnet import resnet50
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena

    torch.manual_seed(0)
    m = resnet50(num_classes=10, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    arena = ParamArena(m)
    arena.enable_bf16_shadow(m)
    return m, arena


def _step(m, arena, xb, yb):
    arena.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(xb)
    F.cross_entropy(out.float(), yb).backward()
    arena.gather_grads()


@gpu
def test_side_stream_wgrad_bitwise(monkeypatch):
    from ray_lightning_accelerators_amd.ops import conv as C

    dev = torch.device("cuda", 0)
    m, arena = _model(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    xb = torch.randn(4, 3, 64, 64, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    yb = torch.randint(0, 10, (4,), device=dev, generator=g)
    monkeypatch.setenv("RLA_WGRAD_STREAM", "0")
    _step(m, arena, xb, yb)  # backend picks (timed) happen here, once
    _step(m, arena, xb, yb)
    ref = arena.grad.clone()
    monkeypatch.setenv("RLA_WGRAD_STREAM", "1")
    n0 = C.side_stats["wgrad"]
    _step(m, arena, xb, yb)
    torch.cuda.synchronize()
    assert C.side_stats["wgrad"] - n0 >= 20  # most layers' weight gradients went to the side stream
    assert torch.equal(arena.grad, ref)


@gpu
def test_side_stream_wgrad_in_graph(monkeypatch):
    dev = torch.device("cuda", 0)
    m, arena = _model(dev)
    g = torch.Generator(device=dev).manual_seed(2)
    xb = torch.randn(4, 3, 64, 64, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    yb = torch.randint(0, 10, (4,), device=dev, generator=g)
    monkeypatch.setenv("RLA_WGRAD_STREAM", "0")
    _step(m, arena, xb, yb)
    _step(m, arena, xb, yb)
    ref = arena.grad.clone()
    monkeypatch.setenv("RLA_WGRAD_STREAM", "1")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _step(m, arena, xb, yb)
    torch.cuda.current_stream().wait_stream(s)
    arena.prepare_graph_capture()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        _step(m, arena, xb, yb)
    arena.grad.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(arena.grad, ref)
