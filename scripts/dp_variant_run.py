"""Run ONE variant of the one-launch MNIST step for a counter pass (rocprofv3 --pmc):
plain (Step1) or a loopback data-parallel protocol at world N.

    python scripts/dp_variant_run.py [--proto packed|owner|none] [--world 1] [--steps 2000]
"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.data import synthetic_mnist  # noqa: E402
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.comm import native_comm_module  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--proto", default="none")
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--steps", type=int, default=2000)
args = ap.parse_args()
dev = torch.device("cuda", 0)
x, y = synthetic_mnist(55000, seed=0)
kw = {}
if args.proto != "none":
    mod = native_comm_module()
    c = mod.Communicator(0, 1, 0)
    c.aux_open([c.aux_handle(fused_mlp.mlp3_dp_capacity(32, 64))])
    base = [int(v) for v in c.aux_context()]
    kw = dict(dp_context=[args.world] + base[1:6] + [base[6]] * args.world, dp_proto=args.proto, dp_loop=True,
              dp_rearm=c.aux_rearm)
eng = FusedMLPEngine(32, 64, 32, lr=1e-3, device=dev, seed=0, **kw)
eng.set_data(x, y)
assert eng.capture(25)
eng.run(args.steps)
torch.cuda.synchronize()
print("ok", args.proto, args.world, float(eng.recent_stats(10)[:, 0].mean()))
