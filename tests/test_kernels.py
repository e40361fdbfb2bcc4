"""Numerics of the HIP kernels vs plain PyTorch fp32 references.

CPU tests exercise the reference implementations (they are the fallback path
and the oracle); ``@pytest.mark.gpu`` tests run the gfx950 kernels and compare
them against torch fp32 on the same data.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from ray_lightning_accelerators_amd import ops
from ray_lightning_accelerators_amd.ops import fused_mlp

gpu = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def _rel(a, b):
    return (a.float() - b.float()).norm().item() / max(b.float().norm().item(), 1e-12)


# ---------------------------------------------------------------- optimizers
def _torch_adam_run(p0, grads, **kw):
    p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p], **kw)
    for g in grads:
        p.grad = g.clone()
        opt.step()
    st = opt.state[p]
    return p.detach(), st["exp_avg"], st["exp_avg_sq"]


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_reference_matches_torch(wd):
    torch.manual_seed(0)
    n = 1037
    p0 = torch.randn(n)
    grads = [torch.randn(n) for _ in range(5)]
    ref_p, ref_m, ref_v = _torch_adam_run(p0, grads, lr=1e-2, weight_decay=wd)
    p, m, v = p0.clone(), torch.zeros(n), torch.zeros(n)
    for t, g in enumerate(grads, 1):
        ops.fused_adam_(p, g, m, v, lr=1e-2, weight_decay=wd, step=t)
    assert torch.allclose(p, ref_p, atol=1e-6, rtol=1e-5)
    assert torch.allclose(m, ref_m, atol=1e-7)
    assert torch.allclose(v, ref_v, atol=1e-7)


@pytest.mark.parametrize("momentum,nesterov,wd", [(0.0, False, 0.0), (0.9, False, 1e-4), (0.9, True, 0.0)])
def test_sgd_reference_matches_torch(momentum, nesterov, wd):
    torch.manual_seed(0)
    n = 515
    p0 = torch.randn(n)
    grads = [torch.randn(n) for _ in range(4)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.SGD([ref], lr=0.1, momentum=momentum, nesterov=nesterov, weight_decay=wd)
    for g in grads:
        ref.grad = g.clone()
        opt.step()
    p, buf = p0.clone(), torch.zeros(n)
    for t, g in enumerate(grads, 1):
        ops.fused_sgd_(p, g, buf, lr=0.1, momentum=momentum, nesterov=nesterov, weight_decay=wd, step=t)
    assert torch.allclose(p, ref.detach(), atol=1e-6)


def test_multi_copy_reference():
    a, b = torch.randn(100), torch.randn(37)
    buf = torch.zeros(137)
    ops.multi_copy([(a, buf[:100]), (b, buf[100:])], scale=0.5)
    assert torch.allclose(buf, torch.cat([a, b]) * 0.5)


def test_mlp_reference_step_matches_autograd():
    torch.manual_seed(0)
    L1, L2, B = 32, 64, 32
    params = fused_mlp.init_mlp_params(L1, L2)
    grads = torch.zeros_like(params)
    x = torch.rand(B, 784)
    y = torch.randint(0, 10, (B,))
    fused_mlp.mlp_train_step(params, grads, L1=L1, L2=L2, B=B, labels=y, x_f32=x)
    model = torch.nn.Sequential(torch.nn.Linear(784, L1), torch.nn.ReLU(), torch.nn.Linear(L1, L2),
                                torch.nn.ReLU(), torch.nn.Linear(L2, 10))
    with torch.no_grad():
        flat = torch.cat([p.reshape(-1) for p in model.parameters()])
        flat.copy_(params)
        off = 0
        for p in model.parameters():
            p.copy_(params[off:off + p.numel()].view_as(p))
            off += p.numel()
    loss = F.nll_loss(F.log_softmax(model(x), 1), y)
    loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    assert _rel(grads, ref) < 1e-5


# ------------------------------------------------------------------ GPU tests
@gpu
def test_native_loaded_on_gpu():
    assert torch.cuda.is_available(), "GPU tests must run on an MI355X box"
    mod = ops.require()
    assert mod.ARCH == "gfx950"
    assert ops.use_native(torch.zeros(1, device=_dev()))


@gpu
@pytest.mark.parametrize("n", [1, 7, 4096, 27882, 1 << 20])
@pytest.mark.parametrize("wd,adamw", [(0.0, False), (0.01, False), (0.01, True)])
def test_adam_native_vs_torch(n, wd, adamw):
    torch.manual_seed(n)
    dev = _dev()
    p0 = torch.randn(n, device=dev)
    grads = [torch.randn(n, device=dev) for _ in range(3)]
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    ref = p0.clone().requires_grad_(True)
    opt = cls([ref], lr=3e-3, weight_decay=wd, foreach=False)
    for g in grads:
        ref.grad = g.clone()
        opt.step()
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    bf = torch.empty(n, dtype=torch.bfloat16, device=dev)
    for g in grads:
        step += 1
        ops.fused_adam_(p, g, m, v, lr=3e-3, weight_decay=wd, adamw=adamw, step=step, p_bf16=bf)
    torch.cuda.synchronize()
    assert torch.allclose(p, ref.detach(), atol=2e-6, rtol=1e-5), (p - ref).abs().max()
    assert torch.equal(bf, p.to(torch.bfloat16))


@gpu
@pytest.mark.parametrize("n", [3, 1000, 65537])
@pytest.mark.parametrize("momentum,nesterov", [(0.0, False), (0.9, False), (0.9, True)])
def test_sgd_native_vs_torch(n, momentum, nesterov):
    torch.manual_seed(1)
    dev = _dev()
    p0 = torch.randn(n, device=dev)
    grads = [torch.randn(n, device=dev) for _ in range(3)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.SGD([ref], lr=0.05, momentum=momentum, nesterov=nesterov, weight_decay=1e-4,
                          foreach=False)
    for g in grads:
        ref.grad = g.clone()
        opt.step()
    p, buf = p0.clone(), torch.zeros_like(p0)
    for t, g in enumerate(grads, 1):
        ops.fused_sgd_(p, g, buf, lr=0.05, momentum=momentum, nesterov=nesterov, weight_decay=1e-4, step=t)
    assert torch.allclose(p, ref.detach(), atol=1e-6, rtol=1e-5)


@gpu
@pytest.mark.parametrize("accumulate", [False, True])
def test_multi_copy_native(accumulate):
    dev = _dev()
    torch.manual_seed(2)
    srcs = [torch.randn(n, device=dev) for n in (1, 5, 16384, 40000, 123)]
    total = sum(s.numel() for s in srcs)
    buf32 = torch.randn(total, device=dev)
    base = buf32.clone()
    pairs, off = [], 0
    for s in srcs:
        pairs.append((s, buf32[off:off + s.numel()]))
        off += s.numel()
    ops.multi_copy(pairs, scale=0.25, accumulate=accumulate)
    exp = torch.cat(srcs) * 0.25 + (base if accumulate else 0)
    assert torch.allclose(buf32, exp, atol=1e-6)
    # fp32 -> bf16 compression and back
    bf = torch.empty(total, dtype=torch.bfloat16, device=dev)
    ops.multi_copy([(buf32, bf)])
    assert torch.equal(bf, buf32.to(torch.bfloat16))
    back = torch.empty(total, device=dev)
    ops.multi_copy([(bf, back)], scale=2.0)
    assert torch.allclose(back, bf.float() * 2.0)


@gpu
def test_scale_sumsq_native():
    dev = _dev()
    x = torch.randn(100003, device=dev)
    ref = (x.double() ** 2).sum().item()
    assert math.isclose(ops.sumsq(x).item(), ref, rel_tol=1e-4)
    y = x.clone()
    ops.scale_(y, 0.125)
    assert torch.allclose(y, x * 0.125)


def _bf(x):
    return x.to(torch.bfloat16).float()


def _emulate_bf16_grads(params, x, y, L1, L2, B):
    """fp32 math with the kernel's bf16 rounding points (the tight oracle)."""
    p = fused_mlp.mlp_unpack(params.cpu(), L1, L2)
    W1, b1, W2, b2, W3, b3 = [p[k] for k in p]
    X = _bf(x)
    h1 = _bf(torch.relu(X @ _bf(W1).T + b1))
    h2 = _bf(torch.relu(h1 @ _bf(W2).T + b2))
    z = h2 @ _bf(W3).T + b3
    pr = torch.softmax(z, 1)
    dz = _bf((pr - F.one_hot(y, 10).float()) / B)
    dh2 = _bf((dz @ _bf(W3)) * (h2 > 0))
    dh1 = _bf((dh2 @ _bf(W2)) * (h1 > 0))
    g = [dh1.T @ X, dh1.sum(0), dh2.T @ h1, dh2.sum(0), dz.T @ h2, dz.sum(0)]
    return torch.cat([t.reshape(-1) for t in g])


def _mlp_case(L1, L2, B, mode, dev, seed=0, n_data=1000):
    g = torch.Generator().manual_seed(seed)
    params = fused_mlp.init_mlp_params(L1, L2, generator=g)
    data = torch.randint(0, 256, (n_data, 784), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, 10, (n_data,), generator=g)
    order = torch.randperm(n_data, generator=g)[: (n_data // B) * B]
    kw = dict(L1=L1, L2=L2, B=B)
    if mode == "u8":
        kw.update(x_u8=data.to(dev), labels=labels.to(dev), order=order.to(dev), n_batches=n_data // B,
                  counters=torch.zeros(2, dtype=torch.int64, device=dev))
    else:
        idx = order[:B]
        kw.update(x_f32=(data[idx].float() / 255.0).to(dev), labels=labels[idx].to(dev),
                  counters=torch.zeros(2, dtype=torch.int64, device=dev))
    return params.to(dev), kw


@gpu
@pytest.mark.parametrize("L1,L2", sorted(fused_mlp.SUPPORTED))
@pytest.mark.parametrize("B", [32, 64, 128])
def test_mlp_grads_native_vs_fp32(L1, L2, B):
    dev = _dev()
    params, kw = _mlp_case(L1, L2, B, "u8", dev)
    grads = torch.zeros_like(params)
    fused_mlp.mlp_train_step(params, grads, **kw)
    # fp32 reference on CPU with the same batch
    cpu_kw = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    cpu_kw["counters"] = torch.zeros(2, dtype=torch.int64)
    ref_g = torch.zeros(params.numel())
    stats = None
    fused_mlp.mlp_train_step(params.cpu(), ref_g, **cpu_kw)
    torch.cuda.synchronize()
    views_n = fused_mlp.mlp_unpack(grads.cpu(), L1, L2)
    views_r = fused_mlp.mlp_unpack(ref_g, L1, L2)
    errs = {name: _rel(views_n[name], views_r[name]) for name in views_n}
    print(f"MLP_FP32_ERR {L1} {L2} {B} " + " ".join(f"{k}={v:.4f}" for k, v in errs.items()))
    # bf16 operands (X, H1, H2, dZ, dH2, dH1) vs an fp32 pipeline: measured at most 0.10
    # norm-wise over every SUPPORTED x B case (profiles/r2_c12/mlp_fp32_err.log), so
    # 0.12 here; plus direction (cosine) -- the tight check follows against the
    # bf16-rounding emulation below
    assert all(e < 0.12 for e in errs.values()), errs
    cos = {n: float(F.cosine_similarity(views_n[n].reshape(1, -1).float(), views_r[n].reshape(1, -1).float()))
           for n in views_n}
    assert all(c > 0.99 for c in cos.values()), cos
    idx = kw["order"][:B].cpu()
    x = kw["x_u8"].cpu()[idx].float() / 255.0
    emu = _emulate_bf16_grads(params, x, kw["labels"].cpu()[idx], L1, L2, B)
    views_e = fused_mlp.mlp_unpack(emu, L1, L2)
    errs_e = {name: _rel(views_n[name], views_e[name]) for name in views_n}
    assert all(e < 1e-2 for e in errs_e.values()), errs_e
    assert kw["counters"][1].item() == 1 and kw["counters"][0].item() == 1
    del stats


@gpu
@pytest.mark.parametrize("B", [1, 17, 48, 100])
def test_mlp_ragged_batch_f32(B):
    dev = _dev()
    L1, L2 = 32, 64
    params, kw = _mlp_case(L1, L2, B, "f32", dev, seed=3)
    grads = torch.zeros_like(params)
    stats = torch.zeros(8, 4, device=dev)
    fused_mlp.mlp_train_step(params, grads, stats=stats, **kw)
    cpu_kw = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    cpu_kw["counters"] = torch.zeros(2, dtype=torch.int64)
    ref_g = torch.zeros(params.numel())
    ref_stats = torch.zeros(8, 4)
    fused_mlp.mlp_train_step(params.cpu(), ref_g, stats=ref_stats, **cpu_kw)
    emu = _emulate_bf16_grads(params, kw["x_f32"].cpu(), kw["labels"].cpu(), L1, L2, B)
    assert _rel(grads.cpu(), emu) < 1e-2
    assert _rel(grads.cpu(), ref_g) < 0.12
    s, rs = stats.cpu()[0], ref_stats[0]
    assert abs(s[0] - rs[0]) < 2e-2 * max(1.0, abs(rs[0]))   # mean loss
    assert abs(s[1] - rs[1]) <= 2                            # correct count
    assert s[2] == B and s[3] == 1


@gpu
@pytest.mark.parametrize("L1,L2,B", [(32, 64, 32), (64, 128, 64), (128, 256, 128)])
def test_mlp_fused_adam_matches_separate(L1, L2, B):
    """apply_adam=True (world size 1) == grads + separate Adam kernel."""
    dev = _dev()
    params, kw = _mlp_case(L1, L2, B, "u8", dev, seed=5)
    p_a = params.clone(); m_a = torch.zeros_like(params); v_a = torch.zeros_like(params)
    p_b = params.clone(); m_b = torch.zeros_like(params); v_b = torch.zeros_like(params)
    g_b = torch.zeros_like(params)
    cnt_a = torch.zeros(2, dtype=torch.int64, device=dev)
    cnt_b = torch.zeros(2, dtype=torch.int64, device=dev)
    for _ in range(3):
        fused_mlp.mlp_train_step(p_a, torch.zeros_like(params), exp_avg=m_a, exp_avg_sq=v_a, apply_adam=True,
                                 lr=1e-2, **{**kw, "counters": cnt_a})
        fused_mlp.mlp_train_step(p_b, g_b, lr=1e-2, **{**kw, "counters": cnt_b})
        ops.fused_adam_(p_b, g_b, m_b, v_b, lr=1e-2, step=cnt_b[0:1])
    torch.cuda.synchronize()
    assert torch.allclose(p_a, p_b, atol=1e-5), (p_a - p_b).abs().max()
    assert cnt_a.tolist() == [3, 3] and cnt_b.tolist() == [3, 3]


@gpu
def test_mlp_eval_native():
    dev = _dev()
    L1, L2, B = 64, 128, 100
    params, kw = _mlp_case(L1, L2, B, "f32", dev, seed=7)
    out = torch.zeros(2, device=dev)
    logits = torch.empty(B, 10, device=dev)
    fused_mlp.mlp_eval(params, L1=L1, L2=L2, B=B, labels=kw["labels"], x_f32=kw["x_f32"], out=out,
                       logits=logits)
    ref_out = torch.zeros(2)
    ref_logits = torch.empty(B, 10)
    fused_mlp.mlp_eval(params.cpu(), L1=L1, L2=L2, B=B, labels=kw["labels"].cpu(), x_f32=kw["x_f32"].cpu(),
                       out=ref_out, logits=ref_logits)
    assert abs(out[0].item() - ref_out[0].item()) < 2e-2 * ref_out[0].item()
    assert abs(out[1].item() - ref_out[1].item()) <= 3
    assert _rel(logits.cpu(), ref_logits) < 2e-2


@gpu
def test_mlp_training_converges_native():
    """A learnable synthetic task: loss must drop well below ln(10)."""
    from ray_lightning_accelerators_amd.models.data import synthetic_mnist

    dev = _dev()
    x, y = synthetic_mnist(4096, seed=0)
    L1, L2, B = 32, 64, 32
    params = fused_mlp.init_mlp_params(L1, L2, torch.Generator().manual_seed(0)).to(dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    nb = 4096 // B
    order = torch.randperm(4096)[: nb * B].to(dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    stats = torch.zeros(256, 4, device=dev)
    for _ in range(200):
        fused_mlp.mlp_train_step(params, torch.zeros_like(params), L1=L1, L2=L2, B=B, labels=y.to(dev),
                                 x_u8=x.to(dev), order=order, counters=cnt, n_batches=nb,
                                 exp_avg=m, exp_avg_sq=v, apply_adam=True, lr=1e-3, stats=stats)
    torch.cuda.synchronize()
    last = stats.cpu()[180:200]
    assert last[:, 0].mean() < 1.0, last[:, 0]


# ------------------------------------------------------- bf16 weight shadows
@gpu
def test_mlp_shadow_refresh_native_matches_reference():
    dev = _dev()
    for L1, L2 in [(32, 64), (128, 256), (64, 128)]:
        p = fused_mlp.init_mlp_params(L1, L2, torch.Generator().manual_seed(L1 + L2)).to(dev)
        lay = fused_mlp.mlp_shadow_layout(L1, L2)
        nat = torch.full((lay["total"],), 7.0, dtype=torch.bfloat16, device=dev)
        nat[lay["w3t"]:] = 0
        fused_mlp.mlp_refresh_shadow(p, nat, L1, L2)
        ref = torch.zeros(lay["total"], dtype=torch.bfloat16)
        fused_mlp.mlp_refresh_shadow(p.cpu(), ref, L1, L2)
        torch.cuda.synchronize()
        assert torch.equal(nat.cpu()[: lay["np"]], ref[: lay["np"]])
        assert torch.equal(nat.cpu()[lay["w2t"]:], ref[lay["w2t"]:])


