"""Resident training loop (csrc/mlp_resident.hip) against the pipelined one-launch
step under hipGraph replays: us/step for windows of K steps, each window bracketed
by device syncs (the bench's timed region).  One JSON line per (mode, K).

  python scripts/resident_probe.py [--reps 5]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)
for mode in ("resident", "graph"):
    eng = FusedMLPEngine(32, 64, 32, lr=1e-3, device=dev, seed=0, resident=(mode == "resident"))
    eng.set_data(x, y)
    if mode == "graph":
        assert eng.capture(20)
    eng.run(100)
    torch.cuda.synchronize()
    for K in (20, 200, 2000):
        best = 1e30
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(K)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"mode": mode, "K": K, "us_per_step": round(best / K * 1e6, 3),
                          "samples_per_s": round(32 * K / best, 1),
                          "loss_last20": round(float(eng.recent_stats(20)[:, 0].mean()), 4)}), flush=True)
