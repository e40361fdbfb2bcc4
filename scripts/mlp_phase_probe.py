"""Diagnostic: per-step wall time of the fused MLP step (v1 single kernel vs v2 head+W1),
plus per-phase timings from in-kernel s_memrealtime stamps (v2 head kernel)."""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device('cuda', 0)
res = {}
x, y = synthetic_mnist(8192, seed=0)
for (L1, L2, B) in [(32, 64, 32), (32, 64, 64), (64, 128, 64), (128, 256, 128)]:
    for ver in (1, 2):
        eng = FusedMLPEngine(L1, L2, B, lr=1e-3, device=dev)
        eng.kernel_version = ver
        eng.set_data(x, y)
        eng.run(50)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run(1000)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 1000 * 1e6
        key = f"{L1}x{L2} B{B} v{ver}"
        entry = {"wall_us_per_step": round(wall, 2)}
        if ver == 2:
            st = torch.zeros(16, dtype=torch.int64, device=dev)
            acc = torch.zeros(6, dtype=torch.float64)
            for _ in range(100):
                fused_mlp.mlp_train_step2(eng.params, eng.grads, shadow=eng.shadow, dh1t=eng.dh1t,
                                          counters=eng.counters, L1=L1, L2=L2, B=B, labels=eng.labels,
                                          x_u8=eng.x_u8, order=eng.order, n_batches=eng.n_batches,
                                          exp_avg=eng.exp_avg, exp_avg_sq=eng.exp_avg_sq, apply_adam=True,
                                          lr=1e-3, stamps=st)
                torch.cuda.synchronize()
                s = st[:6].cpu().double()
                acc += (s - s[0]) * 10.0 / 1000.0
            acc /= 100
            entry["head_phase_end_us"] = dict(zip(["start", "staged", "l1", "l3+softmax", "dH", "end"],
                                                  [round(float(v), 2) for v in acc]))
        res[key] = entry
        print(key, json.dumps(entry), flush=True)
json.dump(res, open('gpurun_out/mlp_phases.json', 'w'), indent=1)
