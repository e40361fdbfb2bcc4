"""Diagnostic: do kernels and the copy engine agree about device memory whose virtual
range was freed back to the driver and mapped again?  (Reading (b) of
docs/one_launch_investigation.md: a stale translation or cache line of a re-used range.)

Per round: tensors of random sizes are written and read by kernels (their translations
and lines get cached), freed and released to the driver (empty_cache), then new tensors
(often at the same addresses) are filled by the copy engine from host patterns -- or
cloned on the device -- and every word is checked twice: an integer checksum reduced by
a kernel against the host pattern's, and a device-to-host copy against the pattern.

    python scripts/remap_stress.py --seconds 120
"""
import argparse
import json
import random
import sys
import time

import torch


def csum(t):
    return int(t.view(torch.int32).long().sum())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = random.Random(11)
    t_end = time.time() + args.seconds
    rounds = checks = bad = reused = 0
    last = time.time()
    while time.time() < t_end:
        sizes = [rng.choice([4096, 16384, 136074, 1 << 18, 1 << 20, 3 << 20]) for _ in range(rng.randint(4, 24))]
        olds = [torch.randn(n, device=dev) * rng.uniform(0.5, 2.0) for n in sizes]
        for t in olds:
            t.mul_(3.0)  # kernel writes
        _ = sum(float(t.sum()) for t in olds)  # kernel reads, on every XCD the grid reaches
        old_ptrs = {t.data_ptr() for t in olds}
        del olds, t
        torch.cuda.synchronize()
        torch.cuda.empty_cache()  # the segments go back to the driver: their ranges are unmapped
        for n in sizes:
            host = torch.randn(n).pin_memory() if rng.random() < 0.5 else torch.randn(n)
            want = csum(host)
            if rng.random() < 0.5:
                d = host.to(dev, non_blocking=True)  # copy engine writes the new range
            else:
                d = host.to(dev).clone()  # ... or a device-side clone of it
            reused += d.data_ptr() in old_ptrs
            got_dev = csum(d)  # the kernels' view
            got_host = csum(d.cpu())  # the copy engine's view
            checks += 1
            if got_dev != want or got_host != want:
                bad += 1
                diff = (d.cpu() != host).nonzero().flatten()
                print(json.dumps({"bad": True, "n": n, "ptr": hex(d.data_ptr()), "reused_addr": d.data_ptr() in old_ptrs,
                                  "dev_ok": got_dev == want, "host_ok": got_host == want,
                                  "host_diff_words": int(diff.numel()),
                                  "first": diff[:4].tolist()}), flush=True)
            del d, host
        rounds += 1
        if time.time() - last > 20:
            print(json.dumps({"progress": rounds, "checks": checks, "bad": bad, "reused": reused}), flush=True)
            last = time.time()
    print(json.dumps({"summary": True, "rounds": rounds, "checks": checks, "bad": bad, "reused_addresses": reused}),
          flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
