"""Split-count sweep of the MFMA weight-gradient kernels (csrc/conv_wgrad.hip): for
each ResNet-50 shape (bs 128), device time of wgrad + its split reduction at the
planner's own S (``auto``) and at fixed S values, so the planner's rule can be
checked against measurements.  One JSON line per shape, then the per-step totals
(weighted by the layer counts) of auto vs the per-shape best.

    python scripts/wgrad_split_sweep.py [--batch 128] [--splits 2,4,8,16,32,64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_lightning_accelerators_amd.ops.conv import _time, wgrad_hip  # noqa: E402
from wgrad_probe import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--splits", default="2,4,8,16,32,64")
    ap.add_argument("--algo", type=int, default=0, help="1: the generic tap-GEMM kernel for every shape")
    ap.add_argument("--kernel", type=int, default=0, help="only shapes with this kernel size (0: all)")
    args = ap.parse_args()
    from ray_lightning_accelerators_amd import ops

    mod = ops.require()
    dev = torch.device("cuda", 0)
    svals = [int(s) for s in args.splits.split(",")]
    tot_auto = tot_best = 0.0
    for (h, cin, cout, k, st, count) in SHAPES:
        if count == 0 or (args.kernel and k != args.kernel):
            continue
        pad = k // 2
        n = args.batch
        oh = (h + 2 * pad - k) // st + 1
        x = torch.randn(n, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, oh, oh, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        auto_plan = list(mod.conv_wgrad_plan(n, h, h, cin, oh, oh, cout, k, k, st, st, pad, pad, 0, args.algo))
        R = 10
        t = {"auto": _time(lambda: wgrad_hip(dy, x, (k, k), (st, st), (pad, pad), 0, args.algo), R) * 1e3 / R}
        for s in svals:
            t[str(s)] = _time(lambda: wgrad_hip(dy, x, (k, k), (st, st), (pad, pad), s, args.algo), R) * 1e3 / R
        best = min(t, key=t.get)
        tot_auto += count * t["auto"]
        tot_best += count * t[best]
        print(json.dumps({"shape": [h, cin, cout, k, st], "count": count, "auto_plan": auto_plan,
                          "us": {a: round(b, 1) for a, b in t.items()}, "best": best}), flush=True)
    print(json.dumps({"per_step_us": {"auto": round(tot_auto, 1), "per_shape_best": round(tot_best, 1)}}), flush=True)


if __name__ == "__main__":
    main()
