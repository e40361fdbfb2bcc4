"""Round-6 deferred-BatchNorm (PRE) kernels against their unfused pairs at ResNet-50's
56x56 stage (batch 128, bf16): the 1x1 forward with statistics (conv3, 64 -> 256), the
3x3 forward with statistics (conv2, 64 -> 64), and the 1x1 / 3x3 weight gradients.

  python scripts/pre_pmc_driver.py --time          # device time per variant (events)
  rocprofv3 --pmc ... -- python3 scripts/pre_pmc_driver.py   # counter passes, 5 reps each

Unfused = bn_apply (relu(x * scale + shift), the materialised activation) + the plain
kernel; fused = the PRE instance reading the BatchNorm's input.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_lightning_accelerators_amd.ops.conv import (  # noqa: E402
    _applied, conv1x1_stats_hip, conv3x3_stats_hip, wgrad_hip)


class _Pre:
    __slots__ = ("st",)

    def __init__(self, st):
        self.st = st

    def take_nbt(self):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, hw, c, c4 = 128, 56, 64, 256
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, c, hw, hw, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    st = torch.stack([torch.zeros(c, device=dev), torch.ones(c, device=dev),
                      torch.rand(c, device=dev, generator=g) + 0.5, torch.randn(c, device=dev, generator=g) * 0.1])
    pre = _Pre(st.contiguous())
    w1 = (torch.randn(c4, c, device=dev, generator=g) / 8).to(torch.bfloat16)
    w3 = (torch.randn(c, c, 3, 3, device=dev, generator=g) / 24).to(torch.bfloat16).contiguous(memory_format=cl)
    dy4 = torch.randn(n, c4, hw, hw, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    dy1 = torch.randn(n, c, hw, hw, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)

    variants = {
        "c1x1_fwd_unfused": lambda: conv1x1_stats_hip(_applied(x, pre), w1),
        "c1x1_fwd_pre": lambda: conv1x1_stats_hip(x, w1, pre),
        "c3x3_fwd_unfused": lambda: conv3x3_stats_hip(_applied(x, pre), w3),
        "c3x3_fwd_pre": lambda: conv3x3_stats_hip(x, w3, pre),
        "wgrad1x1_unfused": lambda: wgrad_hip(dy4, _applied(x, pre), (1, 1), (1, 1), (0, 0)),
        "wgrad1x1_pre": lambda: wgrad_hip(dy4, x, (1, 1), (1, 1), (0, 0), pre_ss=pre.st),
        "wgrad3x3_unfused": lambda: wgrad_hip(dy1, _applied(x, pre), (3, 3), (1, 1), (1, 1)),
        "wgrad3x3_pre": lambda: wgrad_hip(dy1, x, (3, 3), (1, 1), (1, 1), pre_ss=pre.st),
    }
    if not a.time:
        for fn in variants.values():
            for _ in range(a.reps):
                fn()
        torch.cuda.synchronize()
        print("done", flush=True)
        return
    for name, fn in variants.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        best = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best.append(e0.elapsed_time(e1) * 1e3 / 20)
        print(f"{name:20s} {min(best):8.1f} us (median {sorted(best)[2]:.1f})", flush=True)


if __name__ == "__main__":
    main()
