"""Runs only this package's round-5 convolution kernels (no library calls), for
rocprofv3 --pmc passes: the 3x3 forward (plain / with BN statistics) and input
gradient at ResNet-50's four stride-1 shapes, the stem forward (plain / statistics)
and weight gradient.  Batch 128, bf16, 5 reps each.

  rocprofv3 --pmc SQ_WAVES ... -- python3 scripts/kernel_pmc_driver.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_lightning_accelerators_amd.ops.conv import (  # noqa: E402
    conv3x3_dgrad_hip, conv3x3_hip, conv3x3_stats_hip, stem_hip, stem_wgrad_hip)

dev = torch.device("cuda", 0)
n, reps = 128, 5
for hw, c in ((56, 64), (28, 128), (14, 256), (7, 512)):
    x = torch.randn(n, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device=dev) / (3 * c ** 0.5)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    for _ in range(reps):
        conv3x3_hip(x, w)
        conv3x3_stats_hip(x, w)
        conv3x3_dgrad_hip(x, w)
xs = torch.randn(n, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
ws = (torch.randn(64, 3, 7, 7, device=dev) / 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn(n, 64, 112, 112, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for _ in range(reps):
    stem_hip(xs, ws)
    stem_hip(xs, ws, stats=True)
    stem_wgrad_hip(xs, dy)
torch.cuda.synchronize()
print("done", flush=True)
