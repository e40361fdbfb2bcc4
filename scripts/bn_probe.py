"""Achieved HBM bandwidth of the fused BatchNorm kernels (csrc/bn_act.hip) on
ResNet-50's BN shapes (batch 128, NHWC bf16): forward partial / finalize / apply
and the backward partial (y-mask + dy2, writing dres) / apply.  One JSON line per
(shape, kernel): device us per call and GB/s of the bytes the kernel must move.

  python scripts/bn_probe.py [--batch 128] [--reps 20]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.ops import require  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
mod = require()
dev = torch.device("cuda", 0)


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


for hw, c in ((112, 64), (56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024), (7, 512), (7, 2048)):
    n = args.batch
    M = n * hw * hw
    x = torch.randn(M, c, device=dev).to(torch.bfloat16)
    y, dy, dy2, res = (torch.randn_like(x) for _ in range(4))
    out = torch.empty_like(x)
    dres = torch.empty_like(x)
    w = torch.ones(c, device=dev)
    b = torch.zeros(c, device=dev)
    rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
    nbt = torch.zeros((), dtype=torch.long, device=dev)
    part = mod.bn_partial(x, None, None, c, 0, False, nbt)
    st = mod.bn_finalize(part, float(M), w, b, rm, rv, nbt, 0.1, 1e-5)
    bpart = mod.bn_partial(x, y, dy, c, 1, True, None, dy2, None, dres)
    coef = mod.bn_bwd_finalize(bpart, float(M), w, st[0], st[1])
    t = 2.0 * M * c  # bytes of one bf16 tensor
    arms = {
        "fwd_partial": (lambda: mod.bn_partial(x, None, None, c, 0, False, nbt), t),
        "fwd_finalize": (lambda: mod.bn_finalize(part, float(M), w, b, rm, rv, nbt, 0.1, 1e-5), 0.0),
        "fwd_apply_res_relu": (lambda: mod.bn_apply(x, st[2], st[3], res, True, out), 3 * t),
        "fwd_apply_relu": (lambda: mod.bn_apply(x, st[2], st[3], None, True, out), 2 * t),
        "bwd_partial_dy2_wd": (lambda: mod.bn_partial(x, y, dy, c, 1, True, None, dy2, None, dres), 5 * t),
        "bwd_partial_recomp": (lambda: mod.bn_partial(x, None, dy, c, 1, True, None, None, st), 2 * t),
        "bwd_finalize": (lambda: mod.bn_bwd_finalize(bpart, float(M), w, st[0], st[1]), 0.0),
        "bwd_apply_plain": (lambda: mod.bn_bwd_apply(x, None, dres, coef, False, out, None), 3 * t),
        "bwd_apply_recomp": (lambda: mod.bn_bwd_apply(x, None, dy, coef, True, out, None, None, st), 3 * t),
    }
    for name, (fn, nbytes) in arms.items():
        us = timed(fn, args.reps)
        print(json.dumps({"hw": hw, "c": c, "arm": name, "us": round(us, 2),
                          "gb_s": round(nbytes / us * 1e-3, 1) if nbytes else None,
                          "partial_rows": int(part.size(0))}), flush=True)
