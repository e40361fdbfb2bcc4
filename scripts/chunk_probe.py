"""Diagnostic: wall time per step of the fused engine driven the way the Trainer
drives it (dispatch chunks cut at log_every_n_steps = 50 over 1718-batch epochs,
begin_epoch per epoch), with graphs of 25 / 50 steps, with and without the
Trainer's per-chunk host work (row copies + loss/accuracy kernels)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)
B, NB, EVERY = 32, 1718, 50


def epoch(eng, gs, extra):
    order = torch.randperm(55000)[: NB * B]
    eng.begin_epoch(order, NB)
    b = 0
    while b < NB:
        k = min(NB - b, EVERY - gs % EVERY)
        eng.run(k)
        if extra:
            ring = eng.stats.size(0)
            s0 = (gs + k - min(k, ring)) % ring
            n1 = min(k, ring - s0)
            rows = torch.empty(min(k, ring), 4, device=dev)
            rows[:n1].copy_(eng.stats[s0:s0 + n1])
            if n1 < min(k, ring):
                rows[n1:].copy_(eng.stats[: min(k, ring) - n1])
            last = rows[-1]
            _ = last[1] / last[2].clamp(min=1)
            _ = [{"loss": v} for v in rows[:, 0].unbind(0)]
        gs += k
        b += k
    return gs


res = {}
for gsteps in (25, 50):
    for extra in (False, True):
        eng = FusedMLPEngine(32, 64, B, lr=1e-3, device=dev, stats_ring=64)
        eng.attach_dataset(x, y)
        eng.begin_epoch(torch.arange(NB * B), NB)
        eng.capture(gsteps)
        gs = 1
        gs = epoch(eng, gs, extra)  # warm-up epoch (first replays upload the graphs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            gs = epoch(eng, gs, extra)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / (3 * NB) * 1e6
        res[f"graph{gsteps}_{'extra' if extra else 'bare'}"] = round(us, 3)
        print(gsteps, extra, round(us, 3), flush=True)
print(json.dumps(res))
