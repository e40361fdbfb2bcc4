"""Per-shape device time of ResNet-50's convolution weight gradients (bs 128): the
MFMA kernel (csrc/conv_wgrad.hip) vs MIOpen (vs hipBLASLt for the stride-1 1x1s),
with the HBM floor of reading dy and x once.  One JSON line per shape + a summary.

    python scripts/wgrad_probe.py [--batch 128] [--splits 0]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_lightning_accelerators_amd.ops.conv import _time, wgrad_hip  # noqa: E402

# (H_in, Cin, Cout, k, stride, count per step) of ResNet-50 v1.5 with 224x224 input
SHAPES = [
    (56, 64, 64, 1, 1, 1), (56, 64, 256, 1, 1, 3), (56, 256, 64, 1, 1, 2), (56, 256, 128, 1, 1, 1),
    (28, 128, 512, 1, 1, 4), (28, 512, 128, 1, 1, 3), (28, 512, 256, 1, 1, 1),
    (14, 256, 1024, 1, 1, 6), (14, 1024, 256, 1, 1, 5), (14, 1024, 512, 1, 1, 1),
    (7, 512, 2048, 1, 1, 3), (7, 2048, 512, 1, 1, 2),
    (56, 64, 64, 3, 1, 3), (56, 128, 128, 3, 2, 1), (28, 128, 128, 3, 1, 3), (28, 256, 256, 3, 2, 1),
    (14, 256, 256, 3, 1, 5), (14, 512, 512, 3, 2, 1), (7, 512, 512, 3, 1, 2),
    (56, 64, 256, 1, 1, 0), (56, 256, 512, 1, 2, 1), (28, 512, 1024, 1, 2, 1), (14, 1024, 2048, 1, 2, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--splits", type=int, default=0)
    args = ap.parse_args()
    from ray_lightning_accelerators_amd import ops

    mod = ops.require()
    dev = torch.device("cuda", 0)
    tot = {"hip": 0.0, "miopen": 0.0, "best_lib": 0.0, "floor": 0.0}
    for (h, cin, cout, k, st, count) in SHAPES:
        if count == 0:
            continue
        pad = k // 2
        n = args.batch
        oh = (h + 2 * pad - k) // st + 1
        x = torch.randn(n, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, oh, oh, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wb = torch.randn(cout, cin, k, k, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        t = {}
        t["hip"] = _time(lambda: wgrad_hip(dy, x, (k, k), (st, st), (pad, pad), args.splits)) * 1e3 / 3
        t["miopen"] = _time(lambda: torch.ops.aten.convolution_backward(
            dy, x, wb, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])[1].float()) * 1e3 / 3
        if k == 3 and st == 1:
            t["hip_gen"] = _time(lambda: wgrad_hip(dy, x, (k, k), (st, st), (pad, pad), args.splits, 1)) * 1e3 / 3
        if k == 1 and st == 1:
            x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
            d2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            t["gemm"] = _time(lambda: torch.ops.aten.mm.dtype(d2.t(), x2, torch.float32)) * 1e3 / 3
        got = wgrad_hip(dy, x, (k, k), (st, st), (pad, pad), args.splits)
        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), wb.float(), None, [st, st], [pad, pad],
                                                  [1, 1], False, [0, 0], 1, [False, True, False])[1]
        err = float((got - ref).norm() / ref.norm())
        m = n * oh * oh
        in_bytes = 2 * (m * cout + n * h * h * cin)
        floor_us = in_bytes / 5.0e12 * 1e6  # ~5 TB/s achievable HBM read
        plan = mod.conv_wgrad_plan(n, h, h, cin, oh, oh, cout, k, k, st, st, pad, pad, args.splits)
        lib = min(v for key, v in t.items() if not key.startswith("hip"))
        print(json.dumps({"shape": [h, cin, cout, k, st], "count": count, "us": {a: round(b, 1) for a, b in t.items()},
                          "floor_us": round(floor_us, 1), "plan": list(plan), "rel_err": round(err, 7)}), flush=True)
        tot["hip"] += count * min(v for key, v in t.items() if key.startswith("hip"))
        tot["miopen"] += count * t["miopen"]
        tot["best_lib"] += count * lib
        tot["floor"] += count * floor_us
    print(json.dumps({"per_step_us": {a: round(b, 1) for a, b in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
