"""Diagnostic: per-phase timing of the fused MLP step via in-kernel s_memrealtime stamps."""
import sys, time, json
import torch
sys.path.insert(0, '.')
from ray_lightning_accelerators_amd.ops import fused_mlp
from ray_lightning_accelerators_amd.models.data import synthetic_mnist

dev = torch.device('cuda', 0)
names = ["setup", "stage", "l1_mma", "l1_epi", "l2", "l3", "softmax", "dH2", "dH1", "wgrad+adam", "end"]
res = {}
for (L1, L2, B, adam) in [(32, 64, 32, True), (32, 64, 32, False), (64, 128, 64, True), (128, 256, 128, True)]:
    x, y = synthetic_mnist(4096, seed=0)
    params = fused_mlp.init_mlp_params(L1, L2).to(dev)
    g = torch.zeros_like(params); m = torch.zeros_like(params); v = torch.zeros_like(params)
    nb = 4096 // B
    order = torch.randperm(4096)[:nb * B].to(dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    st = torch.zeros(16, dtype=torch.int64, device=dev)
    xs, ys = x.to(dev), y.to(dev)
    kw = dict(L1=L1, L2=L2, B=B, labels=ys, x_u8=xs, order=order, counters=cnt, n_batches=nb,
              exp_avg=m, exp_avg_sq=v, apply_adam=adam, lr=1e-3)
    for _ in range(50):
        fused_mlp.mlp_train_step(params, g, **kw)
    torch.cuda.synchronize()
    acc = torch.zeros(11, dtype=torch.float64)
    N = 200
    for _ in range(N):
        fused_mlp.mlp_train_step(params, g, stamps=st, **kw)
        torch.cuda.synchronize()
        s = st[:11].cpu().double()
        acc += (s - s[0]) * 10.0 / 1000.0  # 100 MHz ticks -> us
    acc /= N
    t0 = time.perf_counter()
    for _ in range(1000):
        fused_mlp.mlp_train_step(params, g, **kw)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 1000 * 1e6
    key = f"{L1}x{L2} B{B} adam={adam}"
    res[key] = {"wall_us_per_step": round(wall, 2),
                "phase_end_us": {n: round(float(a), 2) for n, a in zip(names, acc)}}
    print(key, json.dumps(res[key]))
json.dump(res, open('gpurun_out/mlp_phases.json', 'w'), indent=1)
