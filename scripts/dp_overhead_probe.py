"""Diagnostic: intrinsic cost of the fused data-parallel tail's in-kernel exchange
protocol on ONE GPU.  A world-1 aux region (push to self, then tagged-granule polls
-- or, with RLA_DP_PROTO=wave|all, system fences + flags --
and a fixed-order sum) is driven by the StepDP kernel and timed against the
plain fused step, both replayed from hipGraphs -- a lower bound of what the
exchange adds per step at N > 1 (where the pushes also cross xGMI)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.comm import native_comm_module  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)
mod = native_comm_module()
c = mod.Communicator(0, 1, 0)
c.aux_open([c.aux_handle(2 * fused_mlp.mlp_param_count(32, 64))])  # granule area
ctx = [int(v) for v in c.aux_context()]


def run(kind, n=4000, G=25):
    eng = FusedMLPEngine(32, 64, 32, lr=0.1, device=dev, seed=0)
    eng.set_data(x, y)
    eng.prime()
    kw = eng._kw3()

    def step():
        if kind == "dp":
            fused_mlp.mlp3_launch(fused_mlp.MLP3_STEP_DP, stats=eng.stats, grad_scale=1.0, dp_ctx=ctx, **kw)
        else:
            fused_mlp.mlp3_launch(fused_mlp.MLP3_STEP, stats=eng.stats, **kw)
    for _ in range(50):
        step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(G):
            step()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n // G):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / (n // G * G) * 1e6
    assert c.error_state() == 0, c.error_message()
    return us, float(eng.stats[:, 0].mean())


for rep in range(2):
    for kind in ("plain", "dp"):
        us, loss = run(kind)
        print(f"{kind} us_per_step {us:.2f} loss {loss:.4f}", flush=True)
