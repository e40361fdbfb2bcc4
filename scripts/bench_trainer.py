"""MNISTClassifier throughput through the FULL framework stack: ``Trainer.fit``
with ``RayAccelerator`` (or ``HorovodRayAccelerator``) workers on the local
actor runtime, resident synthetic data, the fused HIP step and (default)
multi-step dispatch -- what a user of the reference's API gets, as opposed to
``bench.py``'s bare engine loop.

Whole-job samples/sec = every rank's training samples over the slowest rank's
epoch time (``ThroughputMonitor``: HIP events at dispatch boundaries).  The
first epoch (allocator, graph capture, RCCL warm-up) is reported, not scored.

    python scripts/bench_trainer.py [--workers 1] [--accelerator ddp|horovod]
        [--epochs 3] [--steps-per-dispatch 64] [--use-gpu 1]
"""
import argparse
import gc
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ray_lightning_accelerators_amd.lightning as pl  # noqa: E402
from ray_lightning_accelerators_amd import HorovodRayAccelerator, RayAccelerator  # noqa: E402
from ray_lightning_accelerators_amd import runtime as ray  # noqa: E402
from ray_lightning_accelerators_amd.models.mnist import MNISTClassifier  # noqa: E402
from ray_lightning_accelerators_amd.utils.metrics import ThroughputMonitor  # noqa: E402


class _Dump(ThroughputMonitor):
    """Also records the cyclic-GC pauses of each epoch (host stalls the monitor's
    HIP-event intervals would otherwise show without a cause)."""

    def __init__(self, path):
        super().__init__()
        self.path = path
        self._gc = []

    def _gc_cb(self, phase, info):
        if phase == "start":
            self._gc_t0 = time.perf_counter()
        else:
            self._gc.append((info.get("generation"), 1e3 * (time.perf_counter() - self._gc_t0)))

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_gc"] = []
        return d

    def on_train_epoch_start(self, trainer, pl_module):
        super().on_train_epoch_start(trainer, pl_module)
        self._gc = []
        if self._gc_cb not in gc.callbacks:
            gc.callbacks.append(self._gc_cb)

    def on_train_epoch_end(self, trainer, pl_module, outputs=None):
        super().on_train_epoch_end(trainer, pl_module, outputs)
        if trainer.global_rank == 0:
            row = dict(self.history[-1], global_step=trainer.global_step,
                       fused=trainer._fused is not None and getattr(trainer._fused, "eng", None) is not None,
                       gc_collections=len(self._gc), gc_ms_max=round(max((t for _, t in self._gc), default=0.0), 3))
            with open(self.path, "a") as f:
                f.write(json.dumps(row) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--accelerator", choices=["ddp", "horovod"], default="ddp")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--layer-1", type=int, default=32)
    ap.add_argument("--layer-2", type=int, default=64)
    ap.add_argument("--steps-per-dispatch", type=int, default=None,
                    help="RLA_STEPS_PER_DISPATCH for the workers (1 = one dispatch per batch)")
    ap.add_argument("--use-gpu", type=int, default=1)
    args = ap.parse_args()
    if args.steps_per_dispatch is not None:
        os.environ["RLA_STEPS_PER_DISPATCH"] = str(args.steps_per_dispatch)
    out = tempfile.mktemp(suffix=".jsonl")
    gpu = bool(args.use_gpu)
    ray.init(num_cpus=2 * args.workers, num_gpus=args.workers if gpu else 0)
    try:
        model = MNISTClassifier({"layer_1": args.layer_1, "layer_2": args.layer_2, "lr": 1e-3,
                                 "batch_size": args.batch_size})
        if args.accelerator == "ddp":
            acc = RayAccelerator(num_workers=args.workers, use_gpu=gpu)
        else:
            acc = HorovodRayAccelerator(num_hosts=1, num_slots=args.workers, use_gpu=gpu)
        trainer = pl.Trainer(default_root_dir=tempfile.mkdtemp(), max_epochs=args.epochs, gpus=int(gpu),
                             limit_val_batches=4, num_sanity_val_steps=0, checkpoint_callback=False,
                             progress_bar_refresh_rate=0, callbacks=[_Dump(out)], accelerator=acc)
        assert trainer.fit(model) == 1
    finally:
        ray.shutdown()
    rows = [json.loads(line) for line in open(out)]
    steady = sorted((rows[1:] or rows), key=lambda r: r.get("samples_per_sec", 0.0))
    best = steady[len(steady) // 2]  # median steady-state epoch
    print(json.dumps({
        "metric": f"samples/sec (whole job), MNISTClassifier Trainer.fit via {type(acc).__name__}",
        "value": round(best.get("samples_per_sec", 0.0), 1), "unit": "samples/s", "workers": args.workers,
        "per_worker_batch": args.batch_size, "use_gpu": gpu, "model": f"784-{args.layer_1}-{args.layer_2}-10",
        "steps_per_dispatch": os.environ.get("RLA_STEPS_PER_DISPATCH", "default"),
        "data": "synthetic", "epochs": rows}), flush=True)


if __name__ == "__main__":
    main()
