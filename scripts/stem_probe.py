"""Device time of ResNet-50's stem convolution (7x7 / stride 2 / pad 3, 3 -> 64,
batch 128, bf16 NHWC): the MFMA stem kernel (csrc/stem.hip) against MIOpen, alone
and with the following BatchNorm's statistics (kernel epilogue vs MIOpen + the BN
partial pass), and the weight gradient.  One JSON line per arm.

  python scripts/stem_probe.py [--batch 128] [--reps 20]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd import ops  # noqa: E402
from ray_lightning_accelerators_amd.ops.conv import stem_hip, stem_wgrad_hip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()

conv = torch.ops.aten.convolution
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True


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


n = args.batch
x = torch.randn(n, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
wb = (torch.randn(64, 3, 7, 7, device=dev) / 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
ref = conv(x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1)
err = float((stem_hip(x, wb).float() - ref.float()).norm() / ref.float().norm())
dy = torch.randn_like(ref)
gref = torch.ops.aten.convolution_backward(dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                           [False, True, False])[1].float()
werr = float((stem_wgrad_hip(x, dy) - gref).norm() / gref.norm())
flop = 2.0 * n * 112 * 112 * 64 * 147
arms = {
    "fwd_miopen": lambda: conv(x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1),
    "fwd_hip": lambda: stem_hip(x, wb),
    "fwd_st_miopen": lambda: ops.require().bn_partial(
        conv(x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1).permute(0, 2, 3, 1), None, None, 64, 0, False,
        None),
    "fwd_st_hip": lambda: stem_hip(x, wb, stats=True),
    "wgrad_miopen": lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0],
                                                               1, [False, True, False])[1],
    "wgrad_hip": lambda: stem_wgrad_hip(x, dy),
}
for name, fn in arms.items():
    us = timed(fn, args.reps)
    print(json.dumps({"arm": name, "batch": n, "us": round(us, 1), "tflops": round(flop / us * 1e-6, 1),
                      "fwd_rel_err_vs_miopen": round(err, 5),
                      "wgrad_rel_err_vs_miopen": round(werr, 5)}), flush=True)
