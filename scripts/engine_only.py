"""Diagnostic: the fused MNIST engine timed alone (no bench / framework imports)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)
eng = FusedMLPEngine(32, 64, 32, lr=0.1, device=dev, seed=0)
eng.set_data(x, y)
eng.capture(8)
eng.run(400)
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    eng.run(4000)
    torch.cuda.synchronize()
    print("engine_only ms_per_step", round((time.perf_counter() - t0) / 4000 * 1e3, 5), flush=True)
