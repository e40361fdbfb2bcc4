"""Host<->device copy integrity under allocator churn (round-6 diagnostic).

Torch-level stress of what the one-launch fidelity test's oracle does between steps:
tensors of the MLP arena's size are produced by kernels on recycled caching-allocator
blocks, copied device->host (``.cpu()``) and host->device (``.to(device)``), and every
copy is checked against a checksum reduced ON the device (8 bytes back).  Any mismatch
means a bulk copy returned / delivered data other than what the device holds.

    python scripts/dma_stress.py --seconds 120 --out gpurun_out/dma_stress.jsonl
"""
from __future__ import annotations

import argparse
import json
import random
import sys
import time

import torch


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = random.Random(7)
    out = open(args.out, "a") if args.out else None
    sizes = [136074, 27882, 59850, 775 * 784 // 4, 100352, 4096, 1 << 20]
    t_end = time.time() + args.seconds
    n = bad = 0
    last = time.time()
    keep = []
    while time.time() < t_end:
        sz = rng.choice(sizes)
        # a kernel-produced tensor on a recycled block
        a = torch.randn(sz, device=dev) * rng.uniform(0.1, 10.0)
        if rng.random() < 0.3:
            b = torch.empty_like(a)
            b.copy_(a)  # device->device
            a = b
        d = int(a.view(torch.int32).long().sum())  # exact: order-independent integer checksum
        h = a.cpu()
        hs = int(h.view(torch.int32).long().sum())
        n += 1
        if hs != d:
            bad += 1
            rec = {"kind": "d2h", "size": sz, "device_sum": d, "host_sum": hs,
                   "host_again": int(a.cpu().view(torch.int32).long().sum()), "ptr": hex(a.data_ptr())}
            print(json.dumps(rec), flush=True)
            if out:
                out.write(json.dumps(rec) + "\n")
        # host->device of fresh host data into a recycled block
        x = torch.randn(sz)
        xd = x.to(dev)
        ds = int(xd.view(torch.int32).long().sum())
        if ds != int(x.view(torch.int32).long().sum()):
            bad += 1
            rec = {"kind": "h2d", "size": sz, "device_sum": ds, "host_sum": int(x.view(torch.int32).long().sum()),
                   "ptr": hex(xd.data_ptr())}
            print(json.dumps(rec), flush=True)
            if out:
                out.write(json.dumps(rec) + "\n")
        keep.append(a)
        if len(keep) > 64:
            keep = keep[rng.randrange(0, 32):]  # free a random batch: churn
        if time.time() - last > 20:
            print(json.dumps({"progress": n, "bad": bad}), flush=True)
            last = time.time()
    summary = {"summary": True, "copies_checked": n, "bad": bad}
    print(json.dumps(summary), flush=True)
    if out:
        out.write(json.dumps(summary) + "\n")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
