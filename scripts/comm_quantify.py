#!/usr/bin/env python
"""Config-5 communication, quantified on ONE GPU.

  buckets     W ranks share the device (gloo bootstrap, native comm engine with the
              xGMI one-shot / two-shot paths over IPC-mapped uncached regions): device
              time of one allreduce per ResNet-50 bucket size {1..25 MiB}, fp32 and
              the bf16 wire, plus the route the router picks.  A PROXY: the "links"
              are this device's own HBM and the W ranks time-slice its CUs, so the
              numbers are a floor for the kernels' own cost, not an xGMI bandwidth.
  trajectory  2 ranks sharing the device train ResNet-50 (bs 32 per rank, a
              learnable synthetic 10-class task) for N steps with the fp32 wire and
              again with the bf16 wire from the same initialisation: per-step losses
              and the final parameter difference.

Usage: python scripts/comm_quantify.py buckets [--world 2] [--reps 20]
       python scripts/comm_quantify.py trajectory [--steps 300]
Rank 0 prints one JSON line per result.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

CAPS_MIB = (1, 2, 4, 8, 16, 25)


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _buckets(rank, world, port, q, reps):
    import torch
    import torch.distributed as dist

    _init(rank, world, port)
    from ray_lightning_accelerators_amd.parallel.comm import NativeCommunicator

    comm = NativeCommunicator(use_rccl=False, use_xgmi=True, xgmi_bytes=2 << 20, twoshot_bytes=64 << 20,
                              spin_limit=1 << 24)
    dev = torch.device("cuda", 0)
    rows = []
    for mib in CAPS_MIB:
        n = mib * (1 << 20) // 4
        x = torch.full((n,), float(rank + 1), device=dev)
        for wire in ("fp32", "bf16"):
            times = []
            for it in range(reps + 3):
                x.fill_(float(rank + 1))
                torch.cuda.synchronize()
                dist.barrier()  # every rank launches together (the kernels poll each other)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                comm.allreduce_(x, bf16_wire=wire == "bf16")
                b.record()
                b.synchronize()
                if it >= 3:
                    times.append(a.elapsed_time(b) * 1e3)
            ok = bool(torch.all(x == world * (world + 1) / 2))
            rows.append({"bucket_mib": mib, "wire": wire, "route": comm.route(x) if wire == "fp32" else "twoshot-bf16",
                         "median_us": round(statistics.median(times), 1), "min_us": round(min(times), 1),
                         "exact": ok})
    comm.check()
    q.put((rank, rows))
    dist.destroy_process_group()


class _Learnable:
    """10-class synthetic images: gaussian noise plus a fixed per-class pattern."""

    def __init__(self, n, size, seed, device):
        import torch

        g = torch.Generator().manual_seed(1234)
        self.protos = (0.5 * torch.randn(10, 3, size, size, generator=g)).to(device)
        g = torch.Generator().manual_seed(seed)
        self.y = torch.randint(0, 10, (n,), generator=g).to(device)
        self.noise = torch.randn(n, 3, size, size, generator=g).to(device)

    def batch(self, i, b):
        import torch

        idx = torch.arange(i * b, (i + 1) * b, device=self.y.device) % self.y.numel()
        x = (self.noise[idx] + self.protos[self.y[idx]]).contiguous(memory_format=torch.channels_last)
        return x, self.y[idx]


def _trajectory(rank, world, port, q, steps, wire, bs, seed=0):
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F

    _init(rank, world, port)
    from ray_lightning_accelerators_amd.models.resnet import resnet50
    from ray_lightning_accelerators_amd.parallel import comm as comm_mod
    from ray_lightning_accelerators_amd.parallel.arena import ParamArena
    from ray_lightning_accelerators_amd.parallel.comm import NativeCommunicator
    from ray_lightning_accelerators_amd.parallel.ddp import GradSynchronizer
    from ray_lightning_accelerators_amd.parallel.fused_optim import fuse_optimizer

    dev = torch.device("cuda", 0)
    # the same kernels in both runs (no per-shape timing that could pick differently):
    # the two trajectories then differ by the gradient wire alone
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    comm_mod._default = NativeCommunicator(use_rccl=False, use_xgmi=True, xgmi_bytes=2 << 20,
                                           twoshot_bytes=64 << 20, spin_limit=1 << 26)
    torch.manual_seed(0)
    model = resnet50(num_classes=10, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    arena = ParamArena(model)
    arena.enable_bf16_shadow(model)
    sync = GradSynchronizer(model, arena, bucket_cap_mb=8.0, grad_dtype=wire, average_in_optimizer=True)
    sync.broadcast_parameters(0)
    # lr 0.1 x (global batch 2 bs / 256), linear warm-up over the first 30 steps
    base_lr = 0.1 * 2 * bs / 256
    sgd = torch.optim.SGD(model.parameters(), lr=base_lr, momentum=0.9, weight_decay=5e-5)
    opt = fuse_optimizer(sgd, arena, grad_scale_fn=lambda: sync.grad_scale)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda i: min(1.0, (i + 1) / 30))
    data = _Learnable(4096, 64, seed=100 + rank + 1000 * seed, device=dev)
    losses = []
    t0 = time.time()
    for i in range(steps):
        x, y = data.batch(i, bs)
        sync.prepare_for_backward()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        sync.finish()
        opt.step()
        opt.zero_grad()
        sched.step()
        losses.append(loss.detach())
    torch.cuda.synchronize()
    comm_mod._default.check()
    flat = arena.data.detach().double().cpu()
    q.put((rank, {"losses": torch.stack(losses).cpu().tolist(), "params": flat, "s": time.time() - t0}))
    dist.destroy_process_group()


def _spawn(target, world, *args):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r, v = q.get(timeout=900)
        out[r] = v
    for p in ps:
        p.join(timeout=60)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["buckets", "trajectory"])
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args(argv)
    if args.what == "buckets":
        out = _spawn(_buckets, args.world, args.reps)
        for i, row in enumerate(out[0]):
            slow = max(out[r][i]["median_us"] for r in out)
            row = dict(row, world=args.world, slowest_rank_median_us=slow,
                       exact=all(out[r][i]["exact"] for r in out), proxy="ranks share one GPU")
            print(json.dumps(row), flush=True)
        return 0
    import torch

    # two data seeds per wire: the fp32-vs-bf16 gap of one seed is judged against the
    # seed-to-seed spread of the SAME wire (training from scratch is chaotic: any
    # difference in the first steps grows into a different trajectory)
    res = {}
    for seed in (0, 1):
        for wire in ("fp32", "bf16"):
            out = _spawn(_trajectory, 2, args.steps, wire, args.batch, seed)
            assert torch.equal(out[0]["params"], out[1]["params"]), "replicas diverged"
            res[wire, seed] = out[0]
            ls = out[0]["losses"]
            print(json.dumps({"wire": wire, "seed": seed, "steps": args.steps, "first_loss": ls[0],
                              "last50_mean_loss": sum(ls[-50:]) / 50, "seconds": round(out[0]["s"], 1),
                              "replicas_equal": True,
                              "losses_every_25": [round(v, 4) for v in ls[::25]]}), flush=True)

    def gap(a, b):
        la, lb = torch.tensor(a["losses"]), torch.tensor(b["losses"])
        return {"mean_abs_loss_diff_last50": round(float((la[-50:] - lb[-50:]).abs().mean()), 4),
                "final_param_rel_diff": round(float((a["params"] - b["params"]).norm() / a["params"].norm()), 4)}

    for seed in (0, 1):
        print(json.dumps(dict(compare=f"bf16 vs fp32 wire, seed {seed}", **gap(res["fp32", seed], res["bf16", seed]))))
    print(json.dumps(dict(compare="fp32 seed 0 vs fp32 seed 1 (natural spread)", **gap(res["fp32", 0], res["fp32", 1]))))
    print(json.dumps(dict(compare="bf16 seed 0 vs bf16 seed 1 (natural spread)", **gap(res["bf16", 0], res["bf16", 1]))))
    return 0


if __name__ == "__main__":
    sys.exit(main())
