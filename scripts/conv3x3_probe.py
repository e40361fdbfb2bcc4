"""Device time of ResNet-50's stride-1 3x3 convolutions (batch 128, bf16, NHWC):
the MFMA kernel (csrc/conv3x3.hip) against MIOpen, forward, forward + BatchNorm
statistics (the kernel's epilogue vs MIOpen + the partial pass) and input gradient.
One JSON line per (shape, op).

  python scripts/conv3x3_probe.py [--batch 128] [--reps 20]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd import ops  # noqa: E402
from ray_lightning_accelerators_amd.ops.conv import conv3x3_dgrad_hip, conv3x3_hip, conv3x3_stats_hip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()

conv = torch.ops.aten.convolution
conv_bwd = torch.ops.aten.convolution_backward
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True  # MIOpen find, as in the model (bench.py)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        torch.cuda._sleep(1_000_000)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / reps)
    return best


for hw, c in ((56, 64), (28, 128), (14, 256), (7, 512)):
    n = args.batch
    x = torch.randn(n, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = (torch.randn(c, c, 3, 3, device=dev) / (3 * c ** 0.5)).to(torch.bfloat16)
    wb = wb.contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    flop = 2.0 * n * hw * hw * c * c * 9
    ref = conv(x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1)
    err = float((conv3x3_hip(x, wb).float() - ref.float()).norm() / ref.float().norm())
    arms = {
        "fwd_miopen": lambda: conv(x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1),
        "fwd_hip": lambda: conv3x3_hip(x, wb),
        # with the next BatchNorm's statistics: the library forward + BN's partial pass
        # vs the kernel's epilogue (what ops.conv picks between for a bn2-feeding conv2)
        "fwd_st_miopen": lambda: ops.require().bn_partial(
            conv(x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1).permute(0, 2, 3, 1), None, None, c, 0,
            False, None),
        "fwd_st_hip": lambda: conv3x3_stats_hip(x, wb),
        "dgrad_miopen": lambda: conv_bwd(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                         [True, False, False])[0],
        "dgrad_hip": lambda: conv3x3_dgrad_hip(dy, wb),
    }
    for name, fn in arms.items():
        us = timed(fn, args.reps)
        print(json.dumps({"hw": hw, "c": c, "batch": n, "arm": name, "us": round(us, 1),
                          "tflops": round(flop / us * 1e-6, 1), "fwd_rel_err_vs_miopen": round(err, 5)}), flush=True)
