"""Diagnostic: in-kernel cost of the one-launch data-parallel step's exchange
protocols on ONE GPU, per world size.

Loopback world N: one process plays all N ranks through its own aux region (the
block writes every source slot itself, polls N granules per value pair, sums;
"owner" also plays every owner: Adam + all-gather publish).  What this prices is
the issue / poll / sum work inside the kernel -- a LOWER bound of what the
exchange adds per step at N ranks, where the pushes also cross xGMI (one hop for
packed, two for owner; see the cost model in csrc/mlp_step3.hip).  Every variant
is replayed from hipGraphs (25 steps per graph) and timed against the plain
one-launch step.  Prints one JSON line per variant.

  python scripts/dp_overhead_probe.py [--steps 4000] [--worlds 1,2,4,8]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.comm import native_comm_module  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=4000)
ap.add_argument("--worlds", default="1,2,4,8")
ap.add_argument("--layers", default="32,64")
args = ap.parse_args()
L1, L2 = (int(v) for v in args.layers.split(","))

dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)
mod = native_comm_module()
c = mod.Communicator(0, 1, 0)
c.aux_open([c.aux_handle(fused_mlp.mlp3_dp_capacity(L1, L2))])
base_ctx = [int(v) for v in c.aux_context()]


def run(proto=None, world=1, G=25):
    kw = {}
    if proto is not None:
        ctx = [world] + base_ctx[1:6] + [base_ctx[6]] * world
        kw = dict(dp_context=ctx, dp_proto=proto, dp_loop=True, dp_rearm=c.aux_rearm)
    eng = FusedMLPEngine(L1, L2, 32, lr=1e-3, device=dev, seed=0, **kw)
    eng.set_data(x, y)
    assert eng.capture(G)
    eng.run(4 * G)
    torch.cuda.synchronize()
    n = args.steps // G * G
    t0 = time.perf_counter()
    eng.run(n)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    assert c.error_state() == 0, c.error_message()
    return us, float(eng.recent_stats(50)[:, 0].mean())


rows = []
for rep in range(2):
    plain, loss = run()
    rows.append({"variant": "plain", "world": 1, "us_per_step": round(plain, 3), "loss": round(loss, 4), "rep": rep})
    print(json.dumps(rows[-1]), flush=True)
    for proto in ("packed", "owner"):
        for w in (int(v) for v in args.worlds.split(",")):
            us, loss = run(proto, w)
            rows.append({"variant": proto, "world": w, "us_per_step": round(us, 3),
                         "overhead_us": round(us - plain, 3), "loss": round(loss, 4), "rep": rep})
            print(json.dumps(rows[-1]), flush=True)
