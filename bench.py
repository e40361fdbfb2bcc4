#!/usr/bin/env python
"""Headline benchmark: MNISTClassifier data-parallel training throughput.

Metric / config come from BASELINE.json: whole-node samples/sec for
MNISTClassifier (MLP 784->32->64->10, Adam, per-worker batch 32 -- the
reference's default config, examples/ray_ddp_example.py:167) at 1/2/4/8
workers, one process per MI355X (torchrun / RayAccelerator worker), RCCL
allreduce over xGMI between ranks.  Weak scaling: per-GPU batch is fixed.

Data: synthetic MNIST-shaped uint8 images + labels (55,000 train samples, the
reference's train split), random-init weights; each rank trains on its
DistributedSampler shard.  Every timed step is a full optimizer step:
forward, NLL loss, backward, gradient allreduce (N > 1), Adam update.

Implementations (``--impl``):
  native  the framework's engine: fused gfx950 HIP step kernel (bf16 MFMA,
          fp32 master weights/Adam), flat-arena allreduce, fused Adam,
          hipGraph replay of the per-step device work.
  torch   stock PyTorch-ROCm baseline: nn.Linear MLP under bf16 autocast,
          torch.optim.Adam, DistributedDataParallel over RCCL (N > 1).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1 is launched by torch.distributed.run, one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "samples/sec (whole node) + DDP scaling eff, MNISTClassifier at 1/2/4/8 workers"
# Our measured stock-PyTorch numbers on MI355X (BASELINE.md "Our MI355X measurements");
# the reference itself publishes none.  None => vs_baseline is null.
RESNET_METRIC = "images/sec (whole node), ResNet-50 synthetic ImageNet 224px"
STOCK_BASELINE = {1: 53015.0}  # --impl torch, 1x MI355X (profiles/r1_first/bench_torch.jsonl)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 2000 (mnist) / 20 (resnet50)")
    ap.add_argument("--warmup", type=int, default=None, help="default 200 (mnist) / 5 (resnet50)")
    ap.add_argument("--model", choices=["mnist", "resnet50"], default="mnist",
                    help="mnist: the BASELINE headline (MNISTClassifier); resnet50: config 5 (bucket stress)")
    ap.add_argument("--impl", choices=["native", "torch"], default="native")
    ap.add_argument("--batch-size", type=int, default=None, help="per GPU; default 32 (mnist) / 128 (resnet50)")
    ap.add_argument("--layer-1", type=int, default=32)
    ap.add_argument("--layer-2", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-1)
    ap.add_argument("--graph-steps", type=int, default=8,
                    help="optimizer steps per captured hipGraph (native); 0 = eager launches")
    ap.add_argument("--n-data", type=int, default=55000)
    ap.add_argument("--bucket-mb", type=float, default=8.0, help="resnet50 DDP bucket cap (MiB)")
    ap.add_argument("--benchmark-algos", type=int, default=1,
                    help="resnet50: torch.backends.cudnn.benchmark (MIOpen find per shape), both impls")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="resnet50 gradient wire dtype (bf16: converted inside the xGMI two-shot kernel)")
    ap.add_argument("--dp", choices=["fused", "split"], default="fused",
                    help="mnist N>1: 'fused' exchanges gradients inside the tail kernel over xGMI "
                         "(falls back to 'split' = head/tail/allreduce/tail when xGMI is unavailable)")
    ap.add_argument("--comm", choices=["auto", "xgmi", "rccl", "torch"], default="auto",
                    help="N>1 gradient allreduce: native xGMI one-shot (auto/xgmi), native RCCL, or c10d")
    args = ap.parse_args()
    rn = args.model == "resnet50"
    if args.steps is None:
        args.steps = 20 if rn else 2000
    if args.warmup is None:
        args.warmup = 5 if rn else 200
    if args.batch_size is None:
        args.batch_size = 128 if rn else 32
    return args


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    if os.environ.get("RLA_BENCH_SHARE_GPU") == "1":
        # rehearsal of the N>1 path on a 1-GPU box: every rank on device 0, gloo
        # bootstrap, native xGMI-protocol allreduce through same-device IPC
        # (throughput is meaningless in this mode; correctness is the point)
        local = 0
        torch.cuda.set_device(0)
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        return world, rank, local
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()


def make_native(args, world, rank, dev, x, y):
    from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine

    allreduce = None
    dp_ctx = None
    if world > 1:
        # native data plane: xGMI one-shot push allreduce for the gradient bucket
        # (validated at setup, RCCL fallback), enqueued on the step's stream so
        # the hipGraph captures it with the step kernels
        from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

        comm = None
        if args.comm != "torch":
            # one 109-532 KiB bucket per step: the one-shot area covers it, so no
            # two-shot region is allocated
            comm = get_native_comm(use_xgmi=args.comm in ("auto", "xgmi"),
                                   use_rccl=dist.get_backend() == "nccl", twoshot_bytes=0)
        if comm is not None:
            if rank == 0:
                print(comm.describe(), file=sys.stderr, flush=True)
            allreduce = comm.allreduce_
            if args.dp == "fused":
                from ray_lightning_accelerators_amd.ops.fused_mlp import mlp_param_count

                dp_ctx = comm.dp_context(mlp_param_count(args.layer_1, args.layer_2))
                if rank == 0:
                    print(f"fused data-parallel tail: {'on' if dp_ctx else 'unavailable (split path)'}",
                          file=sys.stderr, flush=True)
        else:
            allreduce = dist.all_reduce

    eng = FusedMLPEngine(args.layer_1, args.layer_2, args.batch_size, lr=args.lr, device=dev,
                         world_size=world, rank=rank, allreduce=allreduce, seed=0, dp_context=dp_ctx)
    eng.set_data(x, y, shuffle=True)
    eng.broadcast_from(0)
    if args.graph_steps > 0:
        ok = eng.capture(args.graph_steps)
        if not ok and rank == 0:
            print("hipGraph capture failed; running eager", file=sys.stderr)
    def replica_checksum():
        return float(eng.params.double().sum()) + 1e-3 * float(eng.params.double().abs().sum())

    return eng.run, (lambda: float(eng.recent_stats(20)[:, 0].mean())), replica_checksum


def make_torch(args, world, rank, dev, x, y):
    import torch.nn as nn
    import torch.nn.functional as F
    from ray_lightning_accelerators_amd.parallel.mlp_engine import shard_indices

    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(784, args.layer_1), nn.ReLU(), nn.Linear(args.layer_1, args.layer_2),
                          nn.ReLU(), nn.Linear(args.layer_2, 10)).to(dev)
    if world > 1:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    xd, yd = x.to(dev), y.to(dev)
    B = args.batch_size
    state = {"epoch": 0, "i": 0, "last": 0.0}
    per_rank = -(-x.size(0) // world)
    nb = per_rank // B

    def load(epoch):
        state["order"] = shard_indices(x.size(0), world, rank, epoch, 0, True, device=dev)[: nb * B]
        state["i"] = 0

    load(0)

    def run(n):
        for _ in range(n):
            if state["i"] >= nb:
                state["epoch"] += 1
                load(state["epoch"])
            idx = state["order"][state["i"] * B:(state["i"] + 1) * B]
            state["i"] += 1
            xb = xd.index_select(0, idx).float().div_(255.0)
            yb = yd.index_select(0, idx)
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = model(xb)
            loss = F.nll_loss(F.log_softmax(logits.float(), dim=1), yb)
            loss.backward()
            opt.step()
            state["loss"] = loss

    return run, (lambda: float(state["loss"].item()))


def make_resnet(args, world, rank, dev, x, y):
    """ResNet-50, synthetic ImageNet batch resident on the GPU, bf16 autocast, NHWC.

    native: flat fp32 arena + ONE fused SGD-momentum launch, bucketed in-place
    allreduce on the native comm engine's side stream overlapping backward.
    torch:  torch DDP (RCCL) + torch.optim.SGD(foreach)."""
    import torch.nn.functional as F
    from ray_lightning_accelerators_amd.models.resnet import resnet50

    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = bool(args.benchmark_algos)
    # native: BatchNorm+ReLU(+residual add) in the fused gfx950 kernels (ops/bn.py)
    model = resnet50(fused_bn=args.impl == "native").to(dev).to(memory_format=torch.channels_last)
    B = args.batch_size
    g = torch.Generator(device=dev).manual_seed(rank)
    xb = torch.randn(B, 3, 224, 224, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    yb = torch.randint(0, 1000, (B,), device=dev, generator=g)
    state = {}
    if args.impl == "native":
        from ray_lightning_accelerators_amd.parallel.arena import ParamArena
        from ray_lightning_accelerators_amd.parallel.ddp import GradSynchronizer
        from ray_lightning_accelerators_amd.parallel.fused_optim import fuse_optimizer

        arena = ParamArena(model)
        sync = None
        if world > 1:
            from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

            get_native_comm()
            sync = GradSynchronizer(model, arena, bucket_cap_mb=args.bucket_mb, grad_dtype=args.grad_dtype,
                                    average_in_optimizer=True)
            sync.broadcast_parameters(0)
        opt = fuse_optimizer(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5), arena,
                             grad_scale_fn=(lambda: sync.grad_scale) if sync is not None else None)

        def run(n):
            for _ in range(n):
                if sync is not None:
                    sync.prepare_for_backward()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = model(xb)
                loss = F.cross_entropy(out.float(), yb)
                loss.backward()
                if sync is not None:
                    sync.finish()
                opt.step()
                opt.zero_grad()
                state["loss"] = loss
    else:
        m = model
        if world > 1:
            m = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)

        def run(n):
            for _ in range(n):
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = m(xb)
                loss = F.cross_entropy(out.float(), yb)
                loss.backward()
                opt.step()
                state["loss"] = loss

    return run, (lambda: float(state["loss"].item()))


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    from ray_lightning_accelerators_amd.models.data import synthetic_mnist

    if args.model == "resnet50":
        x = y = None
        maker = make_resnet
    else:
        x, y = synthetic_mnist(args.n_data, seed=0)
        maker = make_native if args.impl == "native" else make_torch
    run, last_loss, *extra = maker(args, world, rank, dev, x, y)
    replica_checksum = extra[0] if extra else None

    run(args.warmup)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

        comm = get_native_comm(create=False)
        if comm is not None:
            comm.check()  # a timed-out xGMI poll or RCCL async error invalidates the run
        if replica_checksum is not None:
            # data-parallel replicas must still hold identical weights after the timed steps
            sums = [None] * world
            dist.all_gather_object(sums, replica_checksum())
            if any(v != sums[0] for v in sums):
                raise RuntimeError(f"replicas diverged: {sums}")
    samples = args.steps * args.batch_size * world
    value = samples / elapsed
    loss = last_loss()
    if rank == 0:
        rn = args.model == "resnet50"
        # the stock number is for the default 784-32-64-10 / batch-32 config only
        default_cfg = (args.layer_1, args.layer_2, args.batch_size) == (32, 64, 32)
        base = STOCK_BASELINE.get(world) if (not rn and default_cfg) else None
        out = {
            "metric": RESNET_METRIC if rn else METRIC,
            "value": round(value, 1),
            "unit": "images/s" if rn else "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / base, 3) if base else None),
            "dtype": "bf16",
            "data": "synthetic",
            "config": {
                "model": "ResNet-50" if rn else f"MNISTClassifier(784-{args.layer_1}-{args.layer_2}-10)",
                "global_batch": args.batch_size * world,
                "per_gpu_batch": args.batch_size,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "impl": args.impl,
                "optimizer": "SGD-momentum" if rn else "Adam",
                "final_train_loss": round(loss, 4),
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
