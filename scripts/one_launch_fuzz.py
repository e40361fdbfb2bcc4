"""Fuzz the one-launch MNIST step's first steps (VERDICT r5 item 1 diagnostic).

Engine A runs the one-launch step, engine B the two-launch step (head + tail) from the
same init and data -- the two are bitwise-identical computations
(tests/test_mlp3.py::test_mlp3_one_launch_matches_two_launch), so ANY difference in
A's state after a step is a defect.  Each round builds fresh engines under a random
"session condition":

  plain      nothing else
  garbage    256 MiB of random bits allocated and freed first (the caching allocator
             then hands the engine recycled, dirty memory)
  compute    large GEMMs + convolutions (MIOpen / hipBLASLt) right before each step
             (other kernels' LDS / cache contents on every CU)
  idle       100-400 ms host sleep before each step (the step launches onto an idle GPU)
  loaded     a second process keeps the GPU busy with GEMMs during the whole round

and steps the pair K times with a host sync between steps (as the fidelity test does).
Prints one JSON line per mismatch and a summary line.

    python scripts/one_launch_fuzz.py --seconds 120 --out gpurun_out/fuzz.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

STATE = ("params", "exp_avg", "exp_avg_sq", "shadow", "h1pre", "xring", "yring", "stats")

LOADER = r"""
import sys, time, torch
t_end = time.time() + float(sys.argv[1])
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
while time.time() < t_end:
    for _ in range(20):
        a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
"""


def pollute_garbage(dev):
    g = torch.randint(-2**31, 2**31 - 1, (64 << 20,), dtype=torch.int32, device=dev)
    g.view(torch.float32).add_(0)  # touch as floats too (NaN / Inf patterns included)
    del g


def pollute_compute(dev):
    a = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    for _ in range(4):
        a = (a @ a).clamp_(-3, 3)
    x = torch.randn(32, 64, 56, 56, device=dev, dtype=torch.bfloat16)
    w = torch.randn(64, 64, 3, 3, device=dev, dtype=torch.bfloat16)
    y = F.conv2d(x, w, padding=1)
    y.float().sum().item()


def fp32_ref_grads(flat, xb, yb, L1, L2):
    from ray_lightning_accelerators_amd.ops import fused_mlp

    names = ("W1", "b1", "W2", "b2", "W3", "b3")
    p = {k: v.detach().clone().requires_grad_(True) for k, v in
         zip(names, fused_mlp.mlp_unpack(flat.detach().cpu().float(), L1, L2).values())}
    h = torch.relu(F.linear(xb.float() / 255.0, p["W1"], p["b1"]))
    h = torch.relu(F.linear(h, p["W2"], p["b2"]))
    F.nll_loss(torch.log_softmax(F.linear(h, p["W3"], p["b3"]), 1), yb).backward()
    return {k: p[k].grad for k in names}


BOUND = {"W1": 0.1, "b1": 0.15, "W2": 0.12, "b2": 0.12, "W3": 0.015, "b3": 0.015}


def fidelity(eng, m0, p0, x, y, idx, L1, L2):
    from ray_lightning_accelerators_amd.ops import fused_mlp

    b1 = eng.betas[0]
    g = ((eng.exp_avg - b1 * m0) / (1 - b1)).cpu()
    ref = fp32_ref_grads(p0, x[idx], y[idx], L1, L2)
    out = {}
    for k, v in fused_mlp.mlp_unpack(g, L1, L2).items():
        name = {"layer_1.weight": "W1", "layer_1.bias": "b1", "layer_2.weight": "W2", "layer_2.bias": "b2",
                "layer_3.weight": "W3", "layer_3.bias": "b3"}.get(k, k)
        r = ref[name]
        out[name] = float((v - r).norm() / max(float(r.norm()), 1e-12))
    return out


def one_round(rng, cond, shapes, dev, steps, seed):
    from ray_lightning_accelerators_amd.parallel.mlp_engine import shard_indices

    L1, L2 = rng.choice(shapes)
    B = 32
    x, y = synthetic_mnist(B * rng.choice((6, 12, 24)) + rng.randrange(0, 31), seed=rng.randrange(1000))
    if cond == "garbage":
        pollute_garbage(dev)
    a = FusedMLPEngine(L1, L2, B, lr=1e-3, device=dev, seed=seed)
    b = FusedMLPEngine(L1, L2, B, lr=1e-3, device=dev, seed=seed)
    a.one_launch, b.one_launch = True, False
    a.set_data(x, y)
    b.set_data(x, y)
    for s in range(steps):
        if cond == "compute":
            pollute_compute(dev)
        elif cond == "idle":
            torch.cuda.synchronize()
            time.sleep(rng.uniform(0.1, 0.4))
        epoch, cur = a.epoch, a.step_in_epoch
        idx = shard_indices(x.size(0), 1, 0, epoch, a.seed, True)[cur * B:(cur + 1) * B]
        p0, m0 = a.params.clone(), a.exp_avg.clone()
        a.step()
        b.step()
        torch.cuda.synchronize()
        errs = fidelity(a, m0, p0, x, y, idx, L1, L2)
        if not all(errs[k] < BOUND[k] for k in BOUND):
            return {"mismatch": True, "kind": "fp32", "cond": cond, "L1": L1, "L2": L2, "step": s, "errs": errs,
                    "bitwise_equal_two_launch": all(torch.equal(getattr(a, k), getattr(b, k)) for k in STATE)}
        diff = {k: int((getattr(a, k) != getattr(b, k)).sum()) for k in STATE}
        if any(diff.values()) or not torch.equal(a.counters[:10], b.counters[:10]):
            return {"mismatch": True, "cond": cond, "L1": L1, "L2": L2, "step": s, "diff_elems": diff,
                    "counters_a": a.counters[:11].tolist(), "counters_b": b.counters[:11].tolist(),
                    "hand": a.hand[:17].tolist(), "a_finite": bool(torch.isfinite(a.exp_avg).all()),
                    "b_finite": bool(torch.isfinite(b.exp_avg).all())}
    a.check()
    return {"mismatch": False, "cond": cond, "L1": L1, "L2": L2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--conds", default="plain,garbage,compute,idle,loaded")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = random.Random(1234)
    shapes = [(32, 64), (128, 256), (64, 128)]
    conds = args.conds.split(",")
    counts = {c: [0, 0] for c in conds}
    t_end = time.time() + args.seconds
    out = open(args.out, "a") if args.out else None
    loader = None
    last_print = time.time()
    i = 0
    while time.time() < t_end:
        cond = conds[i % len(conds)]
        if cond == "loaded" and loader is None:
            loader = subprocess.Popen([sys.executable, "-c", LOADER, "20"])
            time.sleep(3.0)  # its first kernels are running
        res = one_round(rng, cond, shapes, dev, args.steps, seed=i)
        if cond == "loaded" and loader is not None and loader.poll() is not None:
            loader = None
        counts[cond][0] += 1
        counts[cond][1] += int(res["mismatch"])
        if res["mismatch"]:
            line = json.dumps(res)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()
        i += 1
        if time.time() - last_print > 30:
            print(json.dumps({"progress": counts}), flush=True)
            last_print = time.time()
    if loader is not None:
        loader.wait(timeout=60)
    summary = {"summary": counts, "rounds": i}
    print(json.dumps(summary), flush=True)
    if out:
        out.write(json.dumps(summary) + "\n")
    return 1 if any(v[1] for v in counts.values()) else 0


if __name__ == "__main__":
    sys.exit(main())
