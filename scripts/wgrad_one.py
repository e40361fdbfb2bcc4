"""Run one weight-gradient kernel configuration repeatedly (for rocprofv3 --pmc passes).

    python scripts/wgrad_one.py --h 56 --cin 64 --cout 64 --k 3 --algo 0 [--reps 50]
"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.ops.conv import wgrad_hip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--h", type=int, default=56)
ap.add_argument("--cin", type=int, default=64)
ap.add_argument("--cout", type=int, default=64)
ap.add_argument("--k", type=int, default=3)
ap.add_argument("--stride", type=int, default=1)
ap.add_argument("--algo", type=int, default=0)
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda", 0)
pad = a.k // 2
oh = (a.h + 2 * pad - a.k) // a.stride + 1
x = torch.randn(a.batch, a.cin, a.h, a.h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn(a.batch, a.cout, oh, oh, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for _ in range(a.reps):
    wgrad_hip(dy, x, (a.k, a.k), (a.stride, a.stride), (pad, pad), 0, a.algo)
torch.cuda.synchronize()
print("ok")
