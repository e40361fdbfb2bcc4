"""Resident MNIST training loop (csrc/mlp_resident.hip): K optimizer steps in one
workgroup of one launch, the model held on one CU.  Checked against an fp32
nn.Linear + torch.optim.Adam run on the same batches (the trajectory bound of the
one-launch step, tests/test_mlp3.py), and for the engine bookkeeping it shares
with the pipelined kernels (counters, stats ring, epoch roll-over, mode switches)."""
import pytest
import torch
import torch.nn.functional as F

from ray_lightning_accelerators_amd.ops import fused_mlp
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine, shard_indices

gpu = pytest.mark.gpu
_NAMES = ("W1", "b1", "W2", "b2", "W3", "b3")


def test_resident_shapes_cpu():
    assert fused_mlp.resident_supported(32, 64, 32)
    assert not fused_mlp.resident_supported(64, 128, 32)
    assert not fused_mlp.resident_supported(32, 64, 64)
    eng = FusedMLPEngine(32, 64, 32, device=torch.device("cpu"))
    assert not eng.resident_ok()  # CPU engine: the reference step


def _reference(x, y, p_init, eng, n, B, lr=1e-3):
    """fp32 torch and stock bf16-autocast trajectories over the engine's batches."""
    L1, L2 = 32, 64
    dev = torch.device("cuda", 0)
    ref = {k: v.clone().requires_grad_(True) for k, v in zip(_NAMES, fused_mlp.mlp_unpack(p_init.cpu(), L1, L2).values())}
    opt = torch.optim.Adam(list(ref.values()), lr=lr)
    ac = {k: v.detach().clone().to(dev).requires_grad_(True) for k, v in ref.items()}
    opt_ac = torch.optim.Adam(list(ac.values()), lr=lr)
    losses = []
    nb = eng.n_batches
    for s in range(n):
        epoch, cur = divmod(s, nb)
        idx = shard_indices(x.size(0), 1, 0, epoch, eng.seed, True)[cur * B:(cur + 1) * B]
        xb = x[idx].float() / 255.0
        h = torch.relu(F.linear(xb, ref["W1"], ref["b1"]))
        h = torch.relu(F.linear(h, ref["W2"], ref["b2"]))
        loss = F.nll_loss(torch.log_softmax(F.linear(h, ref["W3"], ref["b3"]), 1), y[idx])
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            h = torch.relu(F.linear(xb.to(dev), ac["W1"], ac["b1"]))
            h = torch.relu(F.linear(h, ac["W2"], ac["b2"]))
            z = F.linear(h, ac["W3"], ac["b3"])
        loss_ac = F.nll_loss(torch.log_softmax(z.float(), 1), y[idx].to(dev))
        opt_ac.zero_grad()
        loss_ac.backward()
        opt_ac.step()
    p_ref = torch.cat([ref[k].detach().reshape(-1) for k in _NAMES])
    p_ac = torch.cat([ac[k].detach().reshape(-1) for k in _NAMES]).cpu()
    return p_ref, p_ac, losses


@gpu
def test_resident_first_step_matches_fp32_gradient_step():
    """One resident step = one Adam step on bf16 gradients: the parameter update is
    within bf16 compute noise of the fp32 update, per tensor."""
    from ray_lightning_accelerators_amd.models.data import synthetic_mnist

    B = 32
    x, y = synthetic_mnist(B * 20, seed=5)
    eng = FusedMLPEngine(32, 64, B, lr=1e-3, device=torch.device("cuda", 0), seed=1, resident=True)
    eng.set_data(x, y)
    p0 = eng.params.clone()
    assert eng.resident_ok()
    eng.run(1)
    torch.cuda.synchronize()
    p_ref, _, losses = _reference(x, y, p0, eng, 1, B)
    d_k = (eng.params.cpu() - p0.cpu())
    d_r = (p_ref - p0.cpu())
    # Adam's first step moves every weight with a nonzero gradient by ~lr: the signs agree
    for k, a, b in zip(_NAMES, fused_mlp.mlp_unpack(d_k, 32, 64).values(), fused_mlp.mlp_unpack(d_r, 32, 64).values()):
        big = b.abs() > 5e-4
        agree = (torch.sign(a[big]) == torch.sign(b[big])).float().mean().item() if big.any() else 1.0
        assert agree > 0.97, (k, agree)
    assert int(eng.counters[0]) == 1
    st = eng.recent_stats(1)[0]
    assert abs(float(st[0]) - losses[0]) < 2e-2 and int(st[2]) == B and int(st[3]) == 1


@gpu
def test_resident_300_step_trajectory_vs_fp32_torch_adam():
    """300 steps in ONE launch, against fp32 torch Adam fed the same batches from the
    same init (crossing an epoch boundary): the drift stays within 1.5x of what stock
    bf16 autocast drifts and well inside the distance travelled; the loss follows."""
    from ray_lightning_accelerators_amd.models.data import synthetic_mnist

    L1, L2, B, n = 32, 64, 32, 300
    x, y = synthetic_mnist(B * 150, seed=13)
    eng = FusedMLPEngine(L1, L2, B, lr=1e-3, device=torch.device("cuda", 0), seed=3, resident=True)
    eng.set_data(x, y)
    p_init = eng.params.clone()
    eng.run(n)
    torch.cuda.synchronize()
    p_ref, p_ac, losses = _reference(x, y, p_init, eng, n, B)
    p_k = eng.params.cpu()
    moved = (p_ref - p_init.cpu()).norm().item()
    drift = (p_k - p_ref).norm().item() / moved
    drift_ac = (p_ac - p_ref).norm().item() / moved
    loss_k = eng.recent_stats(50)[:, 0].mean().item()
    loss_r = sum(losses[-50:]) / 50
    assert drift < 1.5 * drift_ac + 0.02 and drift < 0.3, (drift, drift_ac)
    assert abs(loss_k - loss_r) < 0.1 * abs(loss_r) + 0.05, (loss_k, loss_r)
    assert int(eng.counters[0]) == n and eng.global_step == n
    rows = eng.recent_stats(n)
    assert torch.equal(rows[:, 3], torch.arange(1, n + 1, dtype=torch.float32))


@gpu
def test_resident_and_pipelined_steps_interleave():
    """run() (resident) and step() (pipelined one-launch) share the engine state:
    counters advance once per step either way, the pipelined kernels re-prime from
    the resident weights (bf16 shadows rebuilt), and training keeps descending."""
    from ray_lightning_accelerators_amd.models.data import synthetic_mnist

    B = 32
    x, y = synthetic_mnist(B * 12, seed=2)
    eng = FusedMLPEngine(32, 64, B, lr=3e-3, device=torch.device("cuda", 0), seed=0, resident=True)
    eng.set_data(x, y)
    eng.run(30)            # resident, crosses two epoch ends (12 batches an epoch)
    for _ in range(5):
        eng.step()         # pipelined
    eng.run(30)
    torch.cuda.synchronize()
    n = 65
    assert int(eng.counters[0]) == n and eng.global_step == n
    assert eng.epoch == n // 12 and eng.step_in_epoch == n % 12
    rows = eng.recent_stats(n)
    assert torch.equal(rows[:, 3], torch.arange(1, n + 1, dtype=torch.float32))
    assert rows[-12:, 0].mean() < rows[:12, 0].mean()
    assert torch.isfinite(eng.params).all()
