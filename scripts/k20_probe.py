"""Where the driver-shaped window (K = 20 steps between two device syncs) loses time
against the steady state: per graph size G (K / G replays) and eager launches, the
median over 50 windows of wall time per step, plus an idle sync round trip and an
empty-graph launch (the fixed costs every window pays).

    python scripts/k20_probe.py [--k 20] [--windows 50]
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
ap.add_argument("--k", type=int, default=20)
ap.add_argument("--windows", type=int, default=50)
ap.add_argument("--sched", choices=["default", "spin", "yield", "blocking"], default="default",
                help="hipSetDeviceFlags scheduling mode, set before the first HIP call")
ap.add_argument("--graphs", default="0,1,2,4,5,10,20")
args = ap.parse_args()
if args.sched != "default":
    import ctypes

    flag = {"spin": 1, "yield": 2, "blocking": 4}[args.sched]
    rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(flag))
    print(json.dumps({"hipSetDeviceFlags": args.sched, "rc": rc}), flush=True)
dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)


def window(run, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(k)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


# fixed costs: an idle synchronize, one tiny kernel + sync
ts = []
for _ in range(200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
z = torch.zeros(1, device=dev)
tk = []
for _ in range(200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    z.add_(1)
    torch.cuda.synchronize()
    tk.append(time.perf_counter() - t0)
print(json.dumps({"idle_sync_us": round(statistics.median(ts) * 1e6, 2),
                  "one_kernel_window_us": round(statistics.median(tk) * 1e6, 2)}), flush=True)

for G in [int(v) for v in args.graphs.split(",")]:
    if G and args.k % G:
        continue
    eng = FusedMLPEngine(32, 64, 32, lr=1e-1, device=dev, seed=0)
    eng.set_data(x, y)
    if G:
        assert eng.capture(G, remainders=False)
        eng.run(G)
    eng.run(2 * args.k)
    w = [window(eng.run, args.k) for _ in range(args.windows)]
    steady = window(eng.run, 2000) / 2000
    print(json.dumps({"graph_steps": G, "k": args.k, "us_per_step_median": round(statistics.median(w) / args.k * 1e6, 3),
                      "us_per_step_min": round(min(w) / args.k * 1e6, 3),
                      "steady_us_per_step": round(steady * 1e6, 3)}), flush=True)
