#!/usr/bin/env python
"""Headline benchmark: MNISTClassifier data-parallel training throughput.

Metric / config come from BASELINE.json: whole-node samples/sec for
MNISTClassifier (MLP 784->32->64->10, Adam, per-worker batch 32 -- the
reference's default config, examples/ray_ddp_example.py:167) at 1/2/4/8
workers, one process per MI355X, gradient allreduce over xGMI between ranks.
Weak scaling: the per-GPU batch is fixed.

Data: synthetic MNIST-shaped uint8 images + labels (55,000 train samples, the
reference's train split), random-init weights; each rank trains on its
DistributedSampler shard.  Every timed step is a full optimizer step:
forward, NLL loss, backward, gradient allreduce (N > 1), Adam update.

Launch (one rank per GPU; the launching process never touches the GPU):
  * ``python bench.py --gpus N`` starts N ``RayExecutor`` actors on the
    framework's runtime -- the workers ``RayAccelerator(num_workers=N,
    use_gpu=True)`` uses, each pinned to its GPU with HIP_VISIBLE_DEVICES
    (reference ray_ddp.py:92-107) -- and prints rank 0's JSON line
    (``--launcher spawn``: N plain child processes that see every GPU, as
    torchrun starts them);
  * ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``:
    every process is one rank (RANK / LOCAL_RANK / WORLD_SIZE from the env).

Implementations (``--impl``):
  native       the framework's engine: fused gfx950 HIP step kernels (bf16
               MFMA, fp32 master weights/Adam), gradient exchange over xGMI
               inside the tail kernel (N > 1), hipGraph replay.
  torch        stock PyTorch-ROCm: nn.Linear MLP under bf16 autocast,
               torch.optim.Adam, DistributedDataParallel over RCCL (N > 1).
  torch-graph  the same stock step captured with torch.cuda.graph (capturable
               Adam, device-side batch cursor), N = 1.

``--via trainer``: the number is ``Trainer.fit`` of ``MNISTClassifier`` through
``RayAccelerator`` (``--accelerator horovod``: ``HorovodRayAccelerator``),
wall-clock over the steady epochs INCLUDING the full validation pass and the
checkpoint write of every epoch (reference examples/ray_ddp_example.py:61-76).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--via engine|trainer]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import subprocess
import sys
import tempfile
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from ray_lightning_accelerators_amd.lightning.callbacks import Callback  # noqa: E402

METRIC = "samples/sec (whole node) + DDP scaling eff, MNISTClassifier at 1/2/4/8 workers"
BENCH_SPIN = 1 << 22  # xGMI poll bound in the bench (~seconds)
RESNET_METRIC = "images/sec (whole node), ResNet-50 synthetic ImageNet 224px"
# Stock PyTorch-ROCm on one MI355X at the default 784-32-64-10 / batch-32 config
# (BASELINE.md "Our MI355X measurements"; the reference publishes no numbers).
# vs_baseline divides by the FASTER stock implementation.
STOCK_BASELINE = {
    "torch": 45378.2,        # eager nn.Linear + torch.optim.Adam (profiles/r3_stock; r1: 53,015)
    "torch-graph": 166204.1,  # the same step under torch.cuda.graph, 8 steps/graph (profiles/r3_stock; r2: 165,417)
}
# ResNet-50 (batch 128, bf16 autocast, channels_last, SGD-momentum) on one MI355X:
# stock torchvision-layout model, eager and under torch.cuda.graph
RESNET_STOCK_BASELINE = {
    "torch": 6010.3,        # profiles/r4_rn/rn50_torch.log
    "torch-graph": 6021.4,  # profiles/r4_rn/rn50_torch_graph.log
}
RESNET_STOCK_SOURCE = {
    "torch": "profiles/r4_rn/rn50_torch.log (round 4, one MI355X, 30 steps)",
    "torch-graph": "profiles/r4_rn/rn50_torch_graph.log (round 4, one MI355X, 30 steps)",
}
# where each hard-coded number was measured (printed in the JSON next to it;
# ``--compare-stock`` re-measures the eager stock step inside the same job)
STOCK_BASELINE_SOURCE = {
    "torch": "profiles/r3_stock/bench_torch.log (round 3 re-measurement, one MI355X, 2000 steps; "
             "round 1: 53,015 in profiles/r1_first/bench_torch.jsonl)",
    "torch-graph": "profiles/r3_stock/bench_torch_graph.log (round 3 re-measurement, one MI355X, 2000 steps; "
                   "round 2: 165,417 in profiles/r2_c03)",
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU; CPU processes with --device cpu)")
    ap.add_argument("--steps", type=int, default=None, help="default 2000 (mnist) / 20 (resnet50)")
    ap.add_argument("--warmup", type=int, default=None, help="default 200 (mnist) / 5 (resnet50)")
    ap.add_argument("--model", choices=["mnist", "resnet50"], default="mnist",
                    help="mnist: the BASELINE headline (MNISTClassifier); resnet50: config 5 (bucket stress)")
    ap.add_argument("--impl", choices=["native", "torch", "torch-graph"], default="native")
    ap.add_argument("--via", choices=["engine", "trainer"], default="engine",
                    help="engine: the worker hot loop; trainer: Trainer.fit through the accelerator")
    ap.add_argument("--accelerator", choices=["ddp", "horovod"], default="ddp",
                    help="ddp: RayAccelerator / DDP process group; horovod: HorovodRayAccelerator / hvd API")
    ap.add_argument("--launcher", choices=["ray", "spawn"], default="ray",
                    help="N>1 without torchrun: runtime actors (GPU-pinned) or plain child processes")
    ap.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto")
    ap.add_argument("--batch-size", type=int, default=None, help="per GPU; default 32 (mnist) / 128 (resnet50)")
    ap.add_argument("--layer-1", type=int, default=32)
    ap.add_argument("--layer-2", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-1)
    ap.add_argument("--graph-steps", type=int, default=8,
                    help="optimizer steps per captured hipGraph (native, torch-graph); 0 = eager launches")
    ap.add_argument("--n-data", type=int, default=55000)
    ap.add_argument("--trainer-epochs", type=int, default=4, help="--via trainer: epochs (the first is warm-up)")
    ap.add_argument("--bucket-mb", type=float, default=8.0, help="resnet50 DDP bucket cap (MiB)")
    ap.add_argument("--bucket-sweep", type=str, default=None,
                    help="resnet50: comma list of bucket caps (MiB) measured in one run, e.g. 1,2,4,8,16,25")
    ap.add_argument("--benchmark-algos", type=int, default=1,
                    help="resnet50: torch.backends.cudnn.benchmark (MIOpen find per shape), both impls")
    ap.add_argument("--resnet-graph", type=int, default=1,
                    help="resnet50 native, 1 GPU: capture the whole training step in one hipGraph (default; "
                         "0 = eager launches, host-bound at ~17 ms/step: profiles/r3_wgrad/rn50_host.log)")
    ap.add_argument("--deterministic-conv", type=int, default=0,
                    help="resnet50: torch.backends.cudnn.deterministic (MIOpen solvers without atomics: no "
                         "zero-fill / cast passes around split-K weight-gradient kernels)")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="resnet50 gradient wire dtype (bf16: converted inside the xGMI two-shot kernel)")
    ap.add_argument("--dp", choices=["fused", "split"], default="fused",
                    help="mnist N>1: 'fused' exchanges gradients inside the step kernel over xGMI (both "
                         "accelerators); 'split' = head/tail/allreduce/tail")
    ap.add_argument("--compare-stock", action="store_true",
                    help="mnist: after the native timing, time the stock step (nn.Linear + torch.optim.Adam, "
                         "torch DDP over RCCL for N > 1) in the same job and report it as stock_*")
    ap.add_argument("--dp-proto", choices=["auto", "packed", "owner", "granule"], default="auto",
                    help="mnist N>1 fused exchange: 'auto' times packed (one-shot) and owner (reduce-scatter / "
                         "owner Adam / all-gather) on this node's links during warm-up and keeps the faster")
    ap.add_argument("--comm", choices=["auto", "xgmi", "rccl", "torch"], default="auto",
                    help="N>1 gradient allreduce: native xGMI (auto/xgmi), native RCCL, or c10d")
    args = ap.parse_args(argv)
    rn = args.model == "resnet50"
    if args.steps is None:
        args.steps = 20 if rn else 2000
    if args.warmup is None:
        args.warmup = 5 if rn else 200
    if args.batch_size is None:
        args.batch_size = 128 if rn else 32
    if args.device == "auto":
        # device_count() does not initialise HIP on this image (the launcher stays GPU-free)
        args.device = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    return args


# ------------------------------------------------------------------ ranks
def rank_env():
    """(world, rank, local) when this process is one rank of a launched job."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"]), int(os.environ.get("LOCAL_RANK", "0"))
    return None


def share_gpu() -> bool:
    # rehearsal of the N>1 path on a 1-GPU box: every rank on device 0, gloo
    # bootstrap, native xGMI-protocol collectives through same-device IPC
    # (throughput is meaningless in this mode; correctness is the point)
    return os.environ.get("RLA_BENCH_SHARE_GPU") == "1"


def setup_dist(args, world, rank, local):
    cpu = args.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
    else:
        if share_gpu() or torch.cuda.device_count() == 1:
            local = 0  # pinned worker (HIP_VISIBLE_DEVICES) or shared device
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        backend = "gloo" if (cpu or share_gpu()) else "nccl"
        kw = {} if backend == "gloo" else {"device_id": dev}
        if args.accelerator == "horovod":
            import ray_lightning_accelerators_amd.horovod as hvd

            os.environ.setdefault("HOROVOD_LOCAL_RANK", str(local))
            if backend == "nccl":
                os.environ["RLA_HVD_USE_GPU"] = "1"
            if backend == "gloo":
                dist.init_process_group("gloo", rank=rank, world_size=world)
            hvd.init()
            assert hvd.size() == world and hvd.rank() == rank
        else:
            dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
    return dev


def barrier(world):
    if world > 1:
        dist.barrier()


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def log(rank, msg):
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


# ----------------------------------------------------------- native engine
def make_native(args, world, rank, dev, x, y, force_split=False):
    from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine

    allreduce = None
    dp_ctx = None
    rearm = None
    route = "single"
    if world > 1:
        from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

        comm = None
        if args.comm != "torch" and dev.type == "cuda":
            # one 109-532 KiB bucket per step: the one-shot area covers it, no two-shot region
            # bench poll bound ~seconds: a step that waits longer for a peer is broken,
            # and the post-capture check below must see it quickly (Trainer runs keep
            # the config's minutes-long bound for peers busy writing checkpoints)
            comm = get_native_comm(use_xgmi=args.comm in ("auto", "xgmi"),
                                   use_rccl=dist.get_backend() == "nccl", twoshot_bytes=0,
                                   spin_limit=BENCH_SPIN)
        if comm is not None:
            log(rank, comm.describe())
            assert comm.world == world
            if args.accelerator == "horovod":
                import ray_lightning_accelerators_amd.horovod as hvd

                allreduce = lambda t: hvd.allreduce_(t, op=hvd.Sum)  # noqa: E731 - hvd API on the native engine
            else:
                allreduce = comm.allreduce_
            if args.dp == "fused" and not force_split:
                from ray_lightning_accelerators_amd.ops.fused_mlp import mlp3_dp_capacity

                dp_ctx = comm.dp_context(mlp3_dp_capacity(args.layer_1, args.layer_2))
                rearm = comm.dp_rearm
            route = "xgmi-fused" if dp_ctx else "split-native"
        else:
            def allreduce(t):
                if t.is_cuda and dist.get_backend() == "gloo":
                    c = t.cpu()
                    dist.all_reduce(c)
                    t.copy_(c)
                else:
                    dist.all_reduce(t)
            route = f"split-c10d-{dist.get_backend()}"
    eng = FusedMLPEngine(args.layer_1, args.layer_2, args.batch_size, lr=args.lr, device=dev,
                         world_size=world, rank=rank, allreduce=allreduce, seed=0, dp_context=dp_ctx,
                         dp_rearm=rearm, dp_proto=None if args.dp_proto == "auto" else args.dp_proto)
    eng.set_data(x, y, shuffle=True)
    eng.broadcast_from(0)
    if route == "split-native":
        from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

        route = f"split-{get_native_comm(create=False).route(eng.comm_buffer)}"  # oneshot / rccl / torch
    graphed = False
    gsteps = graph_steps_for(args.graph_steps, args.steps)
    tuned = None
    if eng.one_launch_dp and args.dp_proto == "auto" and gsteps > 0:
        tuned = tune_dp_proto(eng, world, rank, dev, gsteps)
    if gsteps > 0 and dev.type == "cuda" and route not in ("split-c10d-gloo", "split-torch"):
        graphed = eng.capture(gsteps)
        if graphed:
            # one replay before anything is counted: the first launch of an
            # instantiated graph uploads it (tens of us, once) -- part of capture
            eng.run(gsteps)
        else:
            log(rank, "hipGraph capture failed; running eager launches")

    def replica_checksum():
        return float(eng.params.double().sum()) + 1e-3 * float(eng.params.double().abs().sum())

    one = eng.native and (eng.one_launch_dp if world > 1 else eng.one_launch)
    info = {"route": route, "hip_graph_steps": gsteps if graphed else 0,
            "step_kernel": ("one-launch" if one else "head+tail") if eng.native else "torch-cpu",
            "step_launch": "hip-graph" if graphed else "eager"}
    if eng.dp_ctx is not None:
        info["dp_proto"] = eng.dp_proto
        if tuned is not None:
            info["dp_proto_tuning_us_per_step"] = tuned
    return eng.run, (lambda: float(eng.recent_stats(20)[:, 0].mean())), replica_checksum, info


def tune_dp_proto(eng, world, rank, dev, gsteps, candidates=("packed", "owner"), windows=8):
    """Time each one-launch exchange protocol on THIS node's links (graph replays,
    slowest rank, after a warm replay) and keep the fastest -- the link's small-write
    bandwidth against its hop latency decides between one hop of all the bytes
    (packed) and two hops of 1/N of them (owner); see csrc/mlp_step3.hip.  Every
    rank switches together (collective re-arm of the exchange region).  A protocol
    whose polls time out is discarded.  Returns {proto: us/step}."""
    from ray_lightning_accelerators_amd.parallel.comm import _agree, get_native_comm

    comm = get_native_comm(create=False)
    res = {}
    for name in candidates:
        eng.set_dp_proto(name)
        if not eng.one_launch_dp or not eng.capture(gsteps):
            continue
        eng.run(gsteps)
        t = timed(eng.run, windows * gsteps, world, dev)
        healthy = _agree(comm is None or comm._c.error_state() == 0)
        if not healthy:
            sync(dev)
            barrier(world)
            comm._c.reset_error()
            barrier(world)
            continue
        res[name] = round(t / (windows * gsteps) * 1e6, 3)
    best = min(res, key=res.get) if res else "packed"
    eng.set_dp_proto(best)
    log(rank, f"dp protocol tuning (us/step, slowest rank): {res} -> {best}")
    return res


def degrade_to_split(args, world, rank, dev, x, y):
    """The fused xGMI exchange misbehaved in warm-up (timeout or diverged replicas):
    drop every xGMI path on every rank, clear the latched error and rebuild the
    engine on the split path over RCCL (c10d when RCCL is unavailable)."""
    from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

    comm = get_native_comm(create=False)
    if comm is not None:
        sync(dev)
        barrier(world)
        for path in (0, 1, 2):
            comm._c.disable_path(path)
        comm.xgmi = comm.twoshot = False
        try:
            comm._c.reset_error()
        except RuntimeError:
            pass
        barrier(world)
    log(rank, "fused xGMI data path failed its warm-up check; re-running on the split RCCL path")
    return make_native(args, world, rank, dev, x, y, force_split=True)


def graph_steps_for(requested: int, steps: int) -> int:
    """Steps per captured graph: the largest size <= max(requested, 32) that divides
    the timed step count, so the timed window is whole replays (a 20-step window
    with 8-step graphs would end in 4 eager steps, and every replay's host launch
    is paid once up front)."""
    if requested <= 0:
        return 0
    cap = max(requested, 32)
    for g in range(cap, 0, -1):
        if steps % g == 0:
            return g if g >= min(requested, 4) else requested
    return requested


def replicas_agree(world, checksum) -> bool:
    sums = [None] * world
    dist.all_gather_object(sums, checksum())
    return all(v == sums[0] for v in sums)


def comm_healthy(world) -> bool:
    from ray_lightning_accelerators_amd.parallel.comm import _agree, get_native_comm

    comm = get_native_comm(create=False)
    ok = comm is None or comm._c.error_state() == 0
    return _agree(ok)


# ------------------------------------------------------------ stock torch
def _stock_mlp(args, dev):
    import torch.nn as nn

    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(784, args.layer_1), nn.ReLU(), nn.Linear(args.layer_1, args.layer_2),
                         nn.ReLU(), nn.Linear(args.layer_2, 10)).to(dev)


def make_torch(args, world, rank, dev, x, y):
    import torch.nn.functional as F

    from ray_lightning_accelerators_amd.parallel.mlp_engine import shard_indices

    model = _stock_mlp(args, dev)
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if dev.type == "cuda" else None)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    xd, yd = x.to(dev), y.to(dev)
    B = args.batch_size
    state = {"epoch": 0, "i": 0, "last": 0.0}
    per_rank = -(-x.size(0) // world)
    nb = per_rank // B
    amp = dev.type == "cuda"

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
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                logits = model(xb)
            loss = F.nll_loss(F.log_softmax(logits.float(), dim=1), yb)
            loss.backward()
            opt.step()
            state["loss"] = loss.detach()

    return run, (lambda: float(state["loss"].item())), None, {"route": "torch-ddp" if world > 1 else "single"}


def make_torch_graph(args, world, rank, dev, x, y):
    """Stock step under torch.cuda.graph: capturable Adam, resident data, a device
    batch cursor advanced inside the graph (so replays walk the epoch)."""
    import torch.nn.functional as F

    from ray_lightning_accelerators_amd.parallel.mlp_engine import shard_indices

    if world > 1 or dev.type != "cuda":
        raise SystemExit("--impl torch-graph measures the 1-GPU stock baseline only")
    model = _stock_mlp(args, dev)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr, capturable=True)
    B = args.batch_size
    xd, yd = x.to(dev), y.to(dev)
    nb = x.size(0) // B
    order = shard_indices(x.size(0), 1, 0, 0, 0, True, device=dev)[: nb * B].view(nb, B)
    cursor = torch.zeros((), dtype=torch.int64, device=dev)
    loss_buf = torch.zeros((), device=dev)

    def step():
        idx = order.index_select(0, cursor.view(1)).view(B)
        xb = xd.index_select(0, idx).float().div_(255.0)
        yb = yd.index_select(0, idx)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(xb)
        loss = F.nll_loss(F.log_softmax(logits.float(), dim=1), yb)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        cursor.add_(1).remainder_(nb)
        loss_buf.copy_(loss.detach())

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):  # warm-up outside capture (allocator, autograd state, Adam state)
            step()
    torch.cuda.current_stream().wait_stream(s)
    G = max(1, args.graph_steps)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(G):
            step()

    def run(n):
        for _ in range(n // G):
            g.replay()
        for _ in range(n % G):
            step()

    return run, (lambda: float(loss_buf.item())), None, {"route": "single", "hip_graph_steps": G}


# ----------------------------------------------------------------- ResNet
def make_resnet(args, world, rank, dev, x, y, bucket_mb=None):
    """ResNet-50, synthetic ImageNet batch resident on the GPU, bf16 autocast, NHWC.

    native: flat fp32 arena + ONE fused SGD-momentum launch, bucketed in-place
    allreduce on the native comm engine's side stream overlapping backward.
    torch:  torch DDP (RCCL) + torch.optim.SGD(foreach)."""
    import torch.nn.functional as F

    from ray_lightning_accelerators_amd.models.resnet import resnet50

    if dev.type != "cuda":
        raise SystemExit("--model resnet50 needs a GPU")
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = bool(args.benchmark_algos)
    torch.backends.cudnn.deterministic = bool(args.deterministic_conv)
    # native: BatchNorm+ReLU(+residual add) in the fused gfx950 kernels (ops/bn.py)
    model = resnet50(fused_bn=args.impl == "native").to(dev).to(memory_format=torch.channels_last)
    B = args.batch_size
    g = torch.Generator(device=dev).manual_seed(rank)
    xb = torch.randn(B, 3, 224, 224, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    yb = torch.randint(0, 1000, (B,), device=dev, generator=g)
    state = {}
    info = {"route": "single"}
    if args.impl == "native":
        from ray_lightning_accelerators_amd.parallel.arena import ParamArena
        from ray_lightning_accelerators_amd.parallel.ddp import GradSynchronizer
        from ray_lightning_accelerators_amd.parallel.fused_optim import fuse_optimizer

        arena = ParamArena(model)
        from ray_lightning_accelerators_amd.ops.shadow import wants_shadow

        if wants_shadow(model):
            arena.enable_bf16_shadow(model)  # bf16 weights written by the fused SGD step
        sync_ = None
        if world > 1:
            from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

            comm = get_native_comm()
            if comm is not None:
                log(rank, comm.describe())
            sync_ = GradSynchronizer(model, arena, bucket_cap_mb=bucket_mb or args.bucket_mb,
                                     grad_dtype=args.grad_dtype, average_in_optimizer=True)
            sync_.broadcast_parameters(0)
            info = {"route": "native-reducer", "bucket_mb": bucket_mb or args.bucket_mb}
        opt = fuse_optimizer(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5), arena,
                             grad_scale_fn=(lambda: sync_.grad_scale) if sync_ is not None else None)

        def run(n):
            for _ in range(n):
                if sync_ is not None:
                    sync_.prepare_for_backward()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = model(xb)
                loss = F.cross_entropy(out.float(), yb)
                loss.backward()
                if sync_ is not None:
                    sync_.finish()
                opt.step()
                opt.zero_grad()
                state["loss"] = loss.detach()  # (a live autograd graph must not outlive the step)

        if args.resnet_graph:
            # the whole training step (forward, backward, gradient gather, fused SGD)
            # captured once in a hipGraph and replayed: no per-kernel launch cost for
            # its ~600 kernels.  Capture happens inside the warm-up (after 3 eager
            # steps on a side stream: allocator pools, MIOpen solver choice, the 1x1
            # conv autotune); every replay is one full step on the resident batch.
            # World > 1: the capture also holds the data-parallel part -- the DDP
            # buffer broadcast, every bucket's allreduce forked onto the reducer's
            # comm stream by an event and joined back before the SGD (device-side
            # xGMI generation counters / RCCL: nothing host-side per step).
            eager = run
            gstate = {}

            def run(n):
                if "g" not in gstate:
                    s_ = torch.cuda.Stream()
                    s_.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s_):
                        k = min(3, n)
                        eager(k)
                        n -= k
                    torch.cuda.current_stream().wait_stream(s_)
                    arena.prepare_graph_capture()
                    g_ = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g_):
                        eager(1)
                    gstate["g"] = g_
                for _ in range(n):
                    gstate["g"].replay()

            info = dict(info, hip_graph=True)

        def checksum():
            return float(arena.data.double().sum()) + 1e-3 * float(arena.data.double().abs().sum())
    else:
        m = model
        if world > 1:
            m = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                          bucket_cap_mb=bucket_mb or args.bucket_mb)
            info = {"route": "torch-ddp", "bucket_mb": bucket_mb or args.bucket_mb}
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
        checksum = None

        def run(n):
            for _ in range(n):
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = m(xb)
                loss = F.cross_entropy(out.float(), yb)
                loss.backward()
                opt.step()
                state["loss"] = loss.detach()

        if args.impl == "torch-graph" and world == 1:
            # the fair stock baseline: the same stock step (MIOpen convs /
            # BN, foreach SGD-momentum) captured whole under torch.cuda.graph, so
            # neither side pays per-kernel launch cost.  PyTorch's recipe: warm-up on
            # a side stream (momentum buffers, MIOpen solver choice), grads set to
            # None before the capture, forward + backward + step inside it.
            eager_t = run
            tg = {}

            def run(n):
                if "g" not in tg:
                    s_ = torch.cuda.Stream()
                    s_.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s_):
                        k = min(3, n)
                        eager_t(k)
                        n -= k
                    torch.cuda.current_stream().wait_stream(s_)
                    opt.zero_grad(set_to_none=True)
                    g_ = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g_):
                        with torch.autocast("cuda", dtype=torch.bfloat16):
                            out = m(xb)
                        loss = F.cross_entropy(out.float(), yb)
                        loss.backward()
                        opt.step()
                        state["loss"] = loss.detach()
                    tg["g"] = g_
                for _ in range(n):
                    tg["g"].replay()

            info = dict(info, hip_graph=True)

    return run, (lambda: float(state["loss"].item())), checksum, info


# ------------------------------------------------------------ measurement
def timed(run, steps, world, dev, per_rank=None) -> float:
    """EXACTLY ``steps`` steps, bracketed by barrier + device sync on both sides;
    each rank's clock stops at its own sync (before the closing barrier, whose
    ~50-100 us collective would otherwise be billed to a 20-step window), and the
    slowest rank's time is reported (``per_rank``: list to receive every rank's)."""
    barrier(world)
    sync(dev)
    t0 = time.perf_counter()
    run(steps)
    sync(dev)
    elapsed = time.perf_counter() - t0
    barrier(world)
    if world > 1:
        t = torch.zeros(world, dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        t[dist.get_rank()] = elapsed
        dist.all_reduce(t)  # SUM of one-hot rows = every rank's time
        times = t.cpu().tolist()
        elapsed = max(times)
    else:
        times = [elapsed]
    if per_rank is not None:
        per_rank[:] = times
    return elapsed


def dp_diagnostics(world, per_rank, steps) -> dict:
    """N > 1: what the driver's multi-GPU run should tell a reader:
    per-rank step time, the communicator's bring-up verdict, its RCCL world."""
    us = [t / steps * 1e6 for t in per_rank]
    out = {"per_rank_us_per_step": {"min": round(min(us), 3), "max": round(max(us), 3)}}
    if world > 1:
        from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

        comm = get_native_comm(create=False)
        if comm is not None:
            out["comm"] = comm.describe()
            out["comm_failed_validation"] = list(comm.fallbacks)
            out["rccl_world"] = int(comm._c.rccl_count)
            out["comm_error_state"] = int(comm._c.error_state())
        out["process_group"] = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    return out


def run_rank(args):
    """One rank's measurement; returns rank 0's result dict (None elsewhere)."""
    env = rank_env()
    world, rank, local = env if env is not None else (1, 0, 0)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    dev = setup_dist(args, world, rank, local)
    from ray_lightning_accelerators_amd.models.data import synthetic_mnist

    rn = args.model == "resnet50"
    x = y = None
    if not rn:
        x, y = synthetic_mnist(args.n_data, seed=0)
    maker = {"native": make_native, "torch": make_torch, "torch-graph": make_torch_graph}[args.impl]
    if rn:
        maker = make_resnet
    sweep = None
    if rn and args.bucket_sweep:
        sweep = [float(v) for v in args.bucket_sweep.split(",") if v]
    run, last_loss, checksum, info = maker(args, world, rank, dev, x, y)
    if world > 1 and args.impl == "native" and not rn:
        # self-check of the xGMI data path before anything is timed: the capture ran
        # one real step; a few more, then the error word and replica equality
        run(min(args.warmup, 8))
        sync(dev)
        if not (comm_healthy(world) and replicas_agree(world, checksum)):
            run, last_loss, checksum, info = degrade_to_split(args, world, rank, dev, x, y)
    run(args.warmup)
    log(rank, f"world={world} route={info.get('route')} device={dev}")
    per_rank = []
    elapsed = timed(run, args.steps, world, dev, per_rank)
    diag = dp_diagnostics(world, per_rank, args.steps)
    curve = None
    if sweep:
        curve = {}
        for mb in sweep:
            r2, *_ = make_resnet(args, world, rank, dev, x, y, bucket_mb=mb)
            r2(args.warmup)
            t = timed(r2, args.steps, world, dev)
            curve[str(mb)] = round(args.steps * args.batch_size * world / t, 1)
    if world > 1:
        from ray_lightning_accelerators_amd.parallel.comm import get_native_comm

        comm = get_native_comm(create=False)
        if comm is not None:
            comm.check()  # a timed-out xGMI poll or RCCL async error invalidates the run
        if checksum is not None and not replicas_agree(world, checksum):
            raise RuntimeError("data-parallel replicas diverged after the timed steps")
    n_ranks = dist.get_world_size() if world > 1 else 1
    value = args.steps * args.batch_size * n_ranks / elapsed
    loss = last_loss()
    # fail fast on a diverged / corrupted run: a throughput measured on
    # non-finite training state is not a result
    csum = checksum() if checksum is not None else 0.0
    if not (math.isfinite(loss) and math.isfinite(csum)):
        raise SystemExit(f"bench: non-finite training state after the timed steps "
                         f"(final_train_loss={loss}, parameter checksum={csum})")
    stock = None
    if args.compare_stock and not rn and args.impl == "native" and dev.type == "cuda":
        # the stock stack in the same job, same ranks / data / batch / step count
        # (torch DDP over RCCL for N > 1): both scaling curves from one command
        srun, *_ = make_torch(args, world, rank, dev, x, y)
        srun(min(args.warmup, 50))
        ssteps = min(args.steps, 1000)
        st = timed(srun, ssteps, world, dev)
        stock = {"impl": "torch" + (f"+ddp({dist.get_backend()})" if world > 1 else ""), "steps": ssteps,
                 "value": round(ssteps * args.batch_size * n_ranks / st, 1),
                 "ms_per_step": round(st / ssteps * 1e3, 5)}
    out = None
    if rank == 0:
        default_cfg = (args.layer_1, args.layer_2, args.batch_size) == (32, 64, 32)
        base_impl, base = None, None
        rn_default = rn and args.batch_size == 128 and getattr(args, "impl", "native") == "native"
        if (rn_default or (not rn and default_cfg)) and dev.type == "cuda":
            known = {k: v for k, v in (RESNET_STOCK_BASELINE if rn else STOCK_BASELINE).items() if v}
            if known:
                base_impl = max(known, key=known.get)
                base = known[base_impl]
                if n_ranks > 1:
                    # no stock N-GPU measurement here: the 1-GPU stock number scaled
                    # linearly (an upper bound for stock DDP, so the ratio is conservative)
                    base_impl, base = f"{base_impl} x{n_ranks} (ideal linear)", round(base * n_ranks, 1)
        out = {
            "metric": RESNET_METRIC if rn else METRIC,
            "value": round(value, 1),
            "unit": "images/s" if rn else "samples/s",
            "n_gpus": n_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / base, 3) if base else None),
            "baseline_impl": base_impl,
            "baseline_value": base,
            "baseline_source": (RESNET_STOCK_SOURCE if rn else STOCK_BASELINE_SOURCE).get(
                (base_impl or "").split(" ")[0]),
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": "synthetic",
            "config": {
                "model": "ResNet-50" if rn else f"MNISTClassifier(784-{args.layer_1}-{args.layer_2}-10)",
                "global_batch": args.batch_size * n_ranks,
                "per_gpu_batch": args.batch_size,
                "seq_len": None,
                "parallelism": f"dp{n_ranks}",
                "impl": args.impl,
                "accelerator": args.accelerator,
                "launch": os.environ.get("RLA_BENCH_LAUNCHER", "torchrun" if env is not None else "single"),
                "optimizer": "SGD-momentum" if rn else "Adam",
                "final_train_loss": round(loss, 4),
                **info,
            },
        }
        if rn and args.impl == "native":
            from ray_lightning_accelerators_amd.ops import conv as _conv1x1

            out["conv1x1_backends"] = _conv1x1.choices()
        if world > 1 or args.compare_stock:
            out["dp"] = diag
        if stock:
            out["stock"] = stock
        if curve:
            out["bucket_curve_images_per_s"] = curve
    if world > 1:
        if args.accelerator == "horovod":
            import ray_lightning_accelerators_amd.horovod as hvd

            hvd.shutdown()
        else:
            from ray_lightning_accelerators_amd.parallel.comm import reset_native_comm

            reset_native_comm()
            dist.destroy_process_group()
    return out


# -------------------------------------------------------------- trainer
def _sync_debug() -> None:
    """Print the call stack of each distinct implicit host<->device synchronisation
    (torch's sync debug mode; explicit torch.cuda.synchronize() is not reported)."""
    import traceback
    import warnings

    seen = set()

    def show(msg, cat, filename, lineno, file=None, line=None):
        stack = "".join(traceback.format_stack(limit=10)[:-2])
        if stack not in seen and len(seen) < 30:
            seen.add(stack)
            print(f"[sync-debug] {msg}\n{stack}", file=sys.stderr, flush=True)

    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")


class _EpochClock(Callback):
    """Callback: wall-clock of every epoch from one epoch start to the next (so an
    epoch's time includes its validation pass, checkpoint write and logging),
    max over ranks, plus the per-epoch split train / validation / rest; ``trace``
    also marks every dispatch chunk.  Rank 0 writes the rows to ``path``.

    On the GPU the marks are HIP events recorded on the stream (no host sync: a
    ``synchronize`` per mark stalled the dispatching host at every validation
    start / end and made the measured epoch longer than an unobserved one); the
    interval between two epoch-start events is the epoch's period on the device
    timeline, host stalls included (the device idles while it waits for work)."""

    def __init__(self, path, trace=False):
        self.path = path
        self.trace = trace
        self.marks = []  # (epoch, name, t or event)

    def _mark(self, trainer, name):
        if trainer.on_gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.marks.append((trainer.current_epoch, name, ev))
        else:
            self.marks.append((trainer.current_epoch, name, time.perf_counter()))

    def _resolve(self):
        """Event marks -> seconds on one clock (relative to the first mark)."""
        if not self.marks or not isinstance(self.marks[0][2], torch.cuda.Event):
            return
        torch.cuda.synchronize()
        first = self.marks[0][2]
        self.marks = [(e, n, 0.0 if ev is first else first.elapsed_time(ev) / 1e3) for e, n, ev in self.marks]

    def on_train_epoch_start(self, trainer, pl_module):
        self._mark(trainer, "epoch_start")

    def on_validation_start(self, trainer, pl_module):
        if not trainer.running_sanity_check:
            self._mark(trainer, "val_start")

    def on_validation_end(self, trainer, pl_module):
        if not trainer.running_sanity_check:
            self._mark(trainer, "val_end")

    def on_train_chunk_end(self, trainer, pl_module, outputs, n_steps, n_samples):
        if self.trace:
            self._mark(trainer, "chunk_end")

    def on_train_end(self, trainer, pl_module):
        self._mark(trainer, "train_end")
        self._resolve()
        replicas_equal = None
        arena = getattr(trainer.accelerator_backend, "arena", None)
        if arena is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            # data-parallel replicas after the fit: bitwise-equal parameters on every rank
            cs = float(arena.data.double().sum()) + 1e-3 * float(arena.data.double().abs().sum())
            sums = [None] * dist.get_world_size()
            dist.all_gather_object(sums, cs)
            replicas_equal = all(v == sums[0] for v in sums)
        starts = [t for _, n, t in self.marks if n in ("epoch_start", "train_end")]
        secs = torch.tensor([b - a for a, b in zip(starts, starts[1:])], dtype=torch.float64)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            t = secs.to(trainer.accelerator_backend._comm_device())
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            secs = t.cpu()
        split = []
        for e in range(len(starts) - 1):
            ev = {n: t for ep, n, t in self.marks if ep == e and n in ("val_start", "val_end")}
            t0, t1 = starts[e], starts[e + 1]
            vs, ve = ev.get("val_start", t1), ev.get("val_end", t1)
            row = {"train_s": round(vs - t0, 5), "val_s": round(ve - vs, 5), "rest_s": round(t1 - ve, 5)}
            if self.trace:
                ch = [t for ep, n, t in self.marks if ep == e and n == "chunk_end"]
                gaps = [b - a for a, b in zip([t0] + ch, ch)]
                if gaps:
                    i = max(range(len(gaps)), key=gaps.__getitem__)
                    row.update(chunks=len(gaps), slowest_chunk_s=round(gaps[i], 5), slowest_chunk=i,
                               median_chunk_s=round(statistics.median(gaps), 6))
            split.append(row)
        if trainer.global_rank == 0:
            with open(self.path, "w") as f:
                json.dump({"epoch_s": secs.tolist(), "split": split, "world": trainer.world_size,
                           "clock": "hip-events" if trainer.on_gpu else "host",
                           "batches": int(trainer.num_training_batches),
                           "val_batches": [int(v) for v in trainer.num_val_batches],
                           "fused": trainer._fused is not None,
                           "graph_step": (trainer._fused.describe() if hasattr(trainer._fused, "describe") else
                                          trainer._graph_step_reason),
                           "replicas_equal": replicas_equal,
                           "train_loss": float(trainer.callback_metrics.get(
                               "train_loss", trainer.callback_metrics.get("ptl/train_loss", float("nan")))),
                           "val_loss": float(trainer.callback_metrics.get(
                               "ptl/val_loss", trainer.callback_metrics.get("val_loss", float("nan")))),
                           "val_accuracy": float(trainer.callback_metrics.get(
                               "ptl/val_accuracy", trainer.callback_metrics.get("val_acc", float("nan")))),
                           "best_model_path": getattr(trainer.checkpoint_callback, "best_model_path", None)}, f)


def run_trainer(args):
    """``Trainer.fit(MNISTClassifier)`` through the accelerator; the parent never
    touches the GPU (workers are runtime actors) unless this process is itself a
    torchrun rank (then the env-DDP accelerator runs the same worker flow)."""
    import ray_lightning_accelerators_amd.lightning as pl
    from ray_lightning_accelerators_amd import HorovodRayAccelerator, RayAccelerator
    from ray_lightning_accelerators_amd import runtime as ray
    from ray_lightning_accelerators_amd.models.mnist import MNISTClassifier

    if args.impl != "native":
        raise SystemExit("--via trainer runs the framework path (--impl native)")
    rn = args.model == "resnet50"
    gpu = args.device == "cuda"
    env = rank_env()
    out_path = tempfile.mktemp(prefix="rla-bench-", suffix=".json")
    clock = _EpochClock(out_path, trace=os.environ.get("RLA_BENCH_TRACE") == "1")
    if rn:
        # BASELINE config 5 through the framework: LightningResNet50 on the resident
        # synthetic ImageNet set (`--steps` batches per rank and epoch), the whole step
        # captured by the Trainer (lightning/graph_step.py), a checkpoint every epoch
        from ray_lightning_accelerators_amd.models.resnet import LightningResNet50

        # validation every epoch on a held-out resident set: 2 batches per rank (~10 % of
        # the 20 training steps, the reference MNIST example's 5,000 / 55,000 ratio)
        model = LightningResNet50({"batch_size": args.batch_size, "n_train": args.batch_size * args.steps * args.gpus,
                                   "n_val": args.batch_size * 2 * args.gpus, "lr": 0.1})
    else:
        model = MNISTClassifier({"layer_1": args.layer_1, "layer_2": args.layer_2, "lr": args.lr,
                                 "batch_size": args.batch_size})
    root = tempfile.mkdtemp(prefix="rla-bench-trainer-")
    started = False
    if env is not None:
        acc = "ddp"  # torchrun rank: process group from the env (DDPAccelerator)
        launch = "torchrun"
    else:
        ncpu = max(2, 2 * args.gpus)
        if gpu and share_gpu():
            os.environ["RLA_PG_BACKEND"] = "gloo"  # resolved into the accelerator's config below
            ray.init(num_cpus=ncpu, _nodes=[{"ip": "127.0.0.1", "num_cpus": ncpu, "num_gpus": args.gpus,
                                             "gpu_ids": ["0"] * args.gpus, "resources": {}}])
        else:
            ray.init(num_cpus=ncpu, num_gpus=args.gpus if gpu else 0)
        started = True
        if args.accelerator == "horovod":
            acc = HorovodRayAccelerator(num_hosts=1, num_slots=args.gpus, use_gpu=gpu)
        else:
            acc = RayAccelerator(num_workers=args.gpus, use_gpu=gpu)
        launch = "ray-actors"
    try:
        trainer = pl.Trainer(default_root_dir=root, max_epochs=args.trainer_epochs, gpus=int(gpu),
                             progress_bar_refresh_rate=0, callbacks=[clock], accelerator=acc,
                             benchmark=bool(args.benchmark_algos))
        t0 = time.perf_counter()
        if os.environ.get("RLA_SYNC_DEBUG") == "1" and gpu:
            _sync_debug()  # report every implicit host<->device sync of an in-process fit
        prof_path = os.environ.get("RLA_BENCH_CPROFILE")  # host profile of an in-process fit
        if prof_path:
            import cProfile
            import pstats

            pr = cProfile.Profile()
            pr.enable()
        assert trainer.fit(model) == 1
        fit_s = time.perf_counter() - t0
        if prof_path:
            pr.disable()
            with open(prof_path, "w") as f:
                pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(45)
                # the framework's own functions by cumulative time (per-chunk costs)
                pstats.Stats(pr, stream=f).sort_stats("cumulative").print_stats("ray_lightning_accelerators_amd", 60)
    finally:
        if started:
            ray.shutdown()
    if env is not None and env[1] != 0:
        return None
    with open(out_path) as f:
        rows = json.load(f)
    os.unlink(out_path)
    tl = rows.get("train_loss")
    if tl is None or not math.isfinite(tl):
        raise SystemExit(f"bench: non-finite training loss after Trainer.fit (train_loss={tl})")
    world = rows["world"]
    nb = rows["batches"]
    epochs = rows["epoch_s"]
    steady = epochs[1:] or epochs
    per_epoch = nb * args.batch_size * world
    med = statistics.median(steady)
    value = per_epoch * len(steady) / sum(steady)
    # the same epochs without their validation passes (training + checkpoint only)
    split_steady = rows["split"][1:] or rows["split"]
    no_val_s = sum(max(e - r["val_s"], 1e-9) for e, r in zip(steady, split_steady))
    value_no_val = per_epoch * len(steady) / no_val_s
    if rn:
        base = RESNET_STOCK_BASELINE["torch-graph"] * world
    return {
        "metric": (RESNET_METRIC if rn else METRIC) + " (Trainer.fit wall-clock incl. validation + checkpointing)",
        "value": round(value, 1),
        "unit": "images/s" if rn else "samples/s",
        "n_gpus": world,
        "steps": nb * len(steady),
        "warmup": nb,
        "ms_per_step": round(sum(steady) / (nb * len(steady)) * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / base, 3) if rn and gpu else None,
        "dtype": "bf16" if gpu else "fp32",
        "data": "synthetic" + (" (resident on the device)" if rn else ""),
        "config": {
            "model": "ResNet-50" if rn else f"MNISTClassifier(784-{args.layer_1}-{args.layer_2}-10)",
            "global_batch": args.batch_size * world,
            "per_gpu_batch": args.batch_size,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "via": "trainer",
            "accelerator": type(acc).__name__ if not isinstance(acc, str) else "DDPAccelerator(env)",
            "launch": launch,
            "epochs": args.trainer_epochs,
            "val_batches_per_epoch": rows["val_batches"],
            "train_steps_per_epoch": nb,
            "checkpointing": f"every epoch ({nb} steps)",
            "fused_step": rows["fused"],
            "graph_step": rows.get("graph_step"),
        },
        "replicas_equal": rows.get("replicas_equal"),
        "train_loss": rows.get("train_loss"),
        "epoch_wall_s": [round(v, 5) for v in epochs],
        "epoch_clock": rows.get("clock", "host"),
        "epoch_split": rows["split"],
        "median_steady_epoch_samples_per_s": round(per_epoch / med, 1),
        "steady_epoch_spread": round(max(steady) / min(steady), 3),
        "fit_wall_s": round(fit_s, 2),
        "val_loss": rows["val_loss"],
        "val_accuracy": rows["val_accuracy"],
        "value_without_validation": round(value_no_val, 1),
    }


# --------------------------------------------------------------- launch
def _rank_main(root, argv, rank, world, port, pinned, rla_env):
    """Entry of one rank inside a runtime actor (pickled by value from __main__)."""
    import importlib
    import os as _os
    import sys as _sys

    if root not in _sys.path:
        _sys.path.insert(0, root)
    _os.environ.update(rla_env)  # the launcher's RLA_* knobs (the actor may descend from another env)
    _os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0" if pinned else str(rank),
                        "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                        "RLA_BENCH_LAUNCHER": "ray-actors"})
    bench = importlib.import_module("bench")
    return bench.run_rank(bench.parse(argv))


def launch_ray(args, argv) -> int:
    """N ranks as runtime actors -- the RayAccelerator worker path: RayExecutor
    actors reserving one GPU each (HIP_VISIBLE_DEVICES-pinned), rendezvous port
    chosen on worker 0 (reference ray_ddp.py:92-107, :161-163)."""
    from ray_lightning_accelerators_amd import runtime as ray
    from ray_lightning_accelerators_amd.accelerators.ray_ddp import RayExecutor, find_free_port

    n = args.gpus
    gpu = args.device == "cuda"
    ncpu = n + 1
    if gpu and share_gpu():
        ray.init(num_cpus=ncpu, _nodes=[{"ip": "127.0.0.1", "num_cpus": ncpu, "num_gpus": n,
                                         "gpu_ids": ["0"] * n, "resources": {}}])
    else:
        ray.init(num_cpus=ncpu, num_gpus=n if gpu else 0)
    try:
        workers = [RayExecutor.options(num_cpus=1, num_gpus=int(gpu)).remote() for _ in range(n)]
        port = ray.get(workers[0].execute.remote(find_free_port))
        rla_env = {k: v for k, v in os.environ.items() if k.startswith("RLA_")}
        futures = [w.execute.remote(_rank_main, ROOT, argv, i, n, port, gpu, rla_env) for i, w in enumerate(workers)]
        results = ray.get(futures)
    finally:
        ray.shutdown()
    print(json.dumps(results[0]), flush=True)
    return 0


def launch_spawn(args, argv) -> int:
    """N ranks as plain child processes that see every GPU (torchrun's layout)."""
    from ray_lightning_accelerators_amd.accelerators.ray_ddp import find_free_port

    port = find_free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   RLA_BENCH_LAUNCHER="spawn")
        # intra-op pools sized to each rank's share of the CPUs (N all-core pools oversubscribe)
        env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // args.gpus)))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:  # a failed rank leaves its peers blocked in a collective
                        q.kill()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.via == "trainer":
        res = run_trainer(args)
        if res is not None:
            print(json.dumps(res), flush=True)
        return 0
    if rank_env() is None and args.gpus > 1:
        return launch_ray(args, argv) if args.launcher == "ray" else launch_spawn(args, argv)
    res = run_rank(args)
    if res is not None:
        print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
