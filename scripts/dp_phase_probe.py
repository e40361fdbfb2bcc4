"""Diagnostic: where the one-launch data-parallel step (Step1DP) spends the time it
adds over the plain one-launch step (Step1), from in-kernel s_memrealtime stamps
(100 MHz): block 0's head phases, W1-tile block 1's tail phases and the latest
block end, averaged over 200 eager launches.  Loopback worlds (see
dp_overhead_probe.py) isolate the in-kernel cost of each exchange protocol."""
import json
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.comm import native_comm_module  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device("cuda", 0)
x, y = synthetic_mnist(8192, seed=0)
c = native_comm_module().Communicator(0, 1, 0)
c.aux_open([c.aux_handle(fused_mlp.mlp3_dp_capacity(32, 64))])
base = [int(v) for v in c.aux_context()]
names = ["start", "h1", "l3", "dH", "end", "tiles_end", "small_end", "tile_sx_ready", "tile_start", "tile_head_done",
         "tile_end", "all_end", "heads_end", "last_start", "tile_staged", "tiles_staged"]
VARIANTS = [("plain", None, 1), ("packed", "packed", 1), ("packed", "packed", 8), ("owner", "owner", 8)]
if len(sys.argv) > 1 and sys.argv[1] == "plain":
    VARIANTS = VARIANTS[:1]
for variant, proto, world in VARIANTS:
    kw = {}
    if proto:
        kw = dict(dp_context=[world] + base[1:6] + [base[6]] * world, dp_proto=proto, dp_loop=True,
                  dp_rearm=c.aux_rearm)
    eng = FusedMLPEngine(32, 64, 32, lr=1e-3, device=dev, **kw)
    eng.set_data(x, y)
    eng.run(20)
    # back-to-back launches (the GPU never idles between steps, as in a graph replay),
    # one stamp row per launch, read once at the end
    n = 200
    st = torch.zeros(n, 16, dtype=torch.int64, device=dev)
    k3 = eng._kw3()
    for i in range(n):
        if proto:
            fused_mlp.mlp3_launch(fused_mlp.MLP3_STEP1_DP, stamps=st[i], stats=eng.stats, grad_scale=1.0 / world,
                                  dp_ctx=eng.dp_ctx, dp_proto=fused_mlp.DP_PROTOS[proto], dp_loop=True, **k3)
        else:
            fused_mlp.mlp3_launch(fused_mlp.MLP3_STEP1, stamps=st[i], stats=eng.stats, **k3)
    torch.cuda.synchronize()
    s = st[20:, :16].cpu().double()
    acc = ((s - s[:, :1]) * 10.0 / 1000.0).mean(0)
    period = float((st[21:, 0] - st[20:-1, 0]).double().mean()) * 10.0 / 1000.0
    assert c.error_state() == 0
    print(json.dumps({"variant": variant, "world": world, "launch_period_us": round(period, 3),
                      "phase_us": {k: round(float(v), 3) for k, v in zip(names, acc) if k != "-"}}), flush=True)
