"""Driver for counter passes over the 3x3 MFMA convolution (csrc/conv3x3.hip): each
ResNet-50 stride-1 shape's forward and input gradient, `--reps` times, nothing else
on the GPU in between, so `rocprofv3 --pmc ... -- python scripts/conv3x3_pmc.py`
attributes every conv3x3_kernel dispatch to a shape (dispatch order: per shape,
reps x forward then reps x dgrad).

  python scripts/conv3x3_pmc.py [--batch 128] [--reps 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_lightning_accelerators_amd.ops.conv import conv3x3_dgrad_hip, conv3x3_hip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda", 0)
for hw, c in ((56, 64), (28, 128), (14, 256), (7, 512)):
    x = torch.randn(args.batch, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = (torch.randn(c, c, 3, 3, device=dev) / (3 * c ** 0.5)).to(torch.bfloat16)
    wb = wb.contiguous(memory_format=torch.channels_last)
    for _ in range(args.reps):
        conv3x3_hip(x, wb)
    for _ in range(args.reps):
        conv3x3_dgrad_hip(x, wb)
    torch.cuda.synchronize()
print("done", flush=True)
