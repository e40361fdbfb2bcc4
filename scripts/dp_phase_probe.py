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
names = ["start", "h1", "l3", "dH", "end", "-", "-", "-", "tile_start", "tile_head_done", "tile_end", "all_end"]
for variant, proto, world in [("plain", None, 1), ("packed", "packed", 1), ("packed", "packed", 8),
                              ("owner", "owner", 8)]:
    kw = {}
    if proto:
        kw = dict(dp_context=[world] + base[1:6] + [base[6]] * world, dp_proto=proto, dp_loop=True,
                  dp_rearm=c.aux_rearm)
    eng = FusedMLPEngine(32, 64, 32, lr=1e-3, device=dev, **kw)
    eng.set_data(x, y)
    eng.run(20)
    st = torch.zeros(16, dtype=torch.int64, device=dev)
    acc = torch.zeros(12, dtype=torch.float64)
    k3 = eng._kw3()
    for _ in range(200):
        st.zero_()
        if proto:
            fused_mlp.mlp3_launch(fused_mlp.MLP3_STEP1_DP, stamps=st, stats=eng.stats, grad_scale=1.0 / world,
                                  dp_ctx=eng.dp_ctx, dp_proto=fused_mlp.DP_PROTOS[proto], dp_loop=True, **k3)
        else:
            fused_mlp.mlp3_launch(fused_mlp.MLP3_STEP1, stamps=st, stats=eng.stats, **k3)
        torch.cuda.synchronize()
        s = st[:12].cpu().double()
        acc += (s - s[0]) * 10.0 / 1000.0
    acc /= 200
    assert c.error_state() == 0
    print(json.dumps({"variant": variant, "world": world,
                      "phase_us": {k: round(float(v), 3) for k, v in zip(names, acc) if k != "-"}}), flush=True)
