"""Step-launch mode of the one-launch MNIST step on ONE GPU:
hipGraph replays (G steps per graph) vs back-to-back launches from one C++ call
(FusedMLPEngine.launch_loop), timed exactly like bench.py's window (sync, K steps,
sync) at the driver's K = 20 and at K = 2000.  One JSON line per (mode, K).

  python scripts/launch_mode_probe.py [--reps 7]
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)


def window(eng, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6


for mode, g in (("graph", 20), ("graph", 8), ("loop", 0)):
    eng = FusedMLPEngine(32, 64, 32, lr=1e-1, device=dev, seed=0)
    eng.set_data(x, y, shuffle=True)
    if mode == "loop":
        eng.launch_loop = True
    else:
        assert eng.capture(g)
    eng.run(200)
    for k in (20, 2000):
        us = [window(eng, k) for _ in range(args.reps)]
        print(json.dumps({"mode": mode, "graph_steps": g, "K": k, "us_per_step_median": round(statistics.median(us), 3),
                          "us_per_step_min": round(min(us), 3)}), flush=True)
