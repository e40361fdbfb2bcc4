"""Diagnostic: per-step wall time of the fused MLP step (pipelined head + tail),
eager and hipGraph-replayed, plus per-phase timings of the head kernel (block 0)
and tail block 0 from in-kernel s_memrealtime stamps (100 MHz).  B <= 32 shapes
run both forms: the one-launch step ("one") and head + tail ("two")."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device('cuda', 0)
res = {}
x, y = synthetic_mnist(8192, seed=0)
shapes = [(32, 64, 32), (128, 256, 32), (64, 128, 64), (128, 256, 128)]
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    shapes = shapes[:1]


def wall(eng, n=1000):
    eng.run(50)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(n)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


runs = []
for (L1, L2, B) in shapes:
    if B <= fused_mlp.ONE_LAUNCH_MAX_B:
        runs.append((L1, L2, B, True))
    runs.append((L1, L2, B, False))

for (L1, L2, B, one) in runs:
    eng = FusedMLPEngine(L1, L2, B, lr=1e-3, device=dev)
    eng.one_launch = one
    eng.set_data(x, y)
    entry = {"eager_us_per_step": round(wall(eng), 2)}
    eng.capture(8)
    entry["graph8_us_per_step"] = round(wall(eng), 2)
    st = torch.zeros(16, dtype=torch.int64, device=dev)
    acc = torch.zeros(12, dtype=torch.float64)
    names = ["start", "h1", "l3", "dH", "end", "gather_end", "-", "-", "tail_start", "tail_loaded", "tail_end",
             "tail_all_end"]
    for _ in range(100):
        st.zero_()
        kind = fused_mlp.MLP3_STEP1 if one else fused_mlp.MLP3_STEP
        fused_mlp.mlp3_launch(kind, stamps=st, stats=eng.stats, **eng._kw3())
        torch.cuda.synchronize()
        s = st[:len(names)].cpu().double()
        acc[:len(names)] += (s - s[0]) * 10.0 / 1000.0
    acc /= 100
    entry["phase_end_us"] = {k: round(float(v), 2) for k, v in zip(names, acc) if k != "-"}
    eng.check()
    key = f"{L1}x{L2} B{B}" + (" one" if one else (" two" if B <= fused_mlp.ONE_LAUNCH_MAX_B else ""))
    res[key] = entry
    print(key, json.dumps(entry), flush=True)
json.dump(res, open('gpurun_out/mlp_phases.json', 'w'), indent=1)
