"""Host-side probe of one bench step: enqueue time per phase and host<->device
synchronisations (torch sync-debug mode).  Usage on a GPU box:
    python scripts/step_probe.py --model resnet50 --impl native
"""
import os
import sys
import time
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    x = y = None
    if args.model != "resnet50":
        from ray_lightning_accelerators_amd.models.data import synthetic_mnist

        x, y = synthetic_mnist(args.n_data, seed=0)
    maker = bench.make_resnet if args.model == "resnet50" else (bench.make_native if args.impl == "native"
                                                                 else bench.make_torch)
    run, *_ = maker(args, 1, 0, dev, x, y)
    run(args.warmup)
    torch.cuda.synchronize()
    # enqueue-only timing: how long the host needs to issue one step
    for _ in range(3):
        t0 = time.perf_counter()
        run(1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host enqueue {1e3 * (t1 - t0):.3f} ms, until done {1e3 * (t2 - t0):.3f} ms", flush=True)
    torch.cuda.set_sync_debug_mode("warn")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        run(2)
        torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode(0)
    print(f"synchronising calls in 2 steps: {len(w)}")
    for m in w[:10]:
        print("  ", str(m.message)[:200], m.filename, m.lineno)


if __name__ == "__main__":
    main()
