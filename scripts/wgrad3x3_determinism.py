"""Diagnostic: is the 3x3 halo weight-gradient kernel bitwise reproducible run to run?"""
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
for (n, h, c, co) in [(2, 20, 64, 64), (4, 56, 64, 64), (4, 28, 128, 128), (8, 14, 256, 256), (8, 7, 512, 512)]:
    torch.manual_seed(0)
    x = torch.randn(n, h, h, c, device=dev).to(torch.bfloat16)
    dy = torch.randn(n, h, h, co, device=dev).to(torch.bfloat16)
    res = {}
    for algo in (0, 1):
        outs = [ops.require().conv_wgrad(dy, x, n, h, h, c, h, h, co, 3, 3, 1, 1, 1, 1, 0, algo) for _ in range(6)]
        torch.cuda.synchronize()
        res[algo] = [float((o - outs[0]).abs().max()) for o in outs[1:]]
    print({"shape": (n, h, c, co), "plan": ops.require().conv_wgrad_plan(n, h, h, c, h, h, co, 3, 3, 1, 1, 1, 1, 0, 0),
           "halo_maxdiff": res[0], "generic_maxdiff": res[1]}, flush=True)
