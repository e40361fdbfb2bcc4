"""BASELINE config 1: MNISTClassifier via RayAccelerator(num_workers=2, use_gpu=False)
on the local runtime (CPU / gloo plumbing).  Whole-job samples/sec of the
training epochs as measured by ThroughputMonitor inside the workers.

    python scripts/bench_cpu_plumbing.py [--workers 2] [--batches 200] [--epochs 2]
"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ray_lightning_accelerators_amd.lightning as pl  # noqa: E402
from ray_lightning_accelerators_amd import RayAccelerator  # noqa: E402
from ray_lightning_accelerators_amd import runtime as ray  # noqa: E402
from ray_lightning_accelerators_amd.models.mnist import MNISTClassifier  # noqa: E402
from ray_lightning_accelerators_amd.utils.metrics import ThroughputMonitor  # noqa: E402


class _Dump(ThroughputMonitor):
    def __init__(self, path):
        super().__init__()
        self.path = path

    def on_train_epoch_end(self, trainer, pl_module, outputs=None):
        super().on_train_epoch_end(trainer, pl_module, outputs)
        if trainer.global_rank == 0:
            with open(self.path, "a") as f:
                f.write(json.dumps(self.history[-1]) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch-size", type=int, default=32)
    args = ap.parse_args()
    out = tempfile.mktemp(suffix=".jsonl")
    ray.init(num_cpus=args.workers, num_gpus=0)
    try:
        model = MNISTClassifier({"layer_1": 32, "layer_2": 64, "lr": 1e-3, "batch_size": args.batch_size})
        trainer = pl.Trainer(default_root_dir=tempfile.mkdtemp(), max_epochs=args.epochs,
                             limit_train_batches=args.batches, limit_val_batches=1, checkpoint_callback=False,
                             progress_bar_refresh_rate=0, callbacks=[_Dump(out)],
                             accelerator=RayAccelerator(num_workers=args.workers, use_gpu=False))
        assert trainer.fit(model) == 1
    finally:
        ray.shutdown()
    rows = [json.loads(line) for line in open(out)]
    last = rows[-1]  # the first epoch includes gloo / allocator warm-up
    print(json.dumps({"metric": "samples/sec (whole job), MNISTClassifier RayAccelerator CPU/gloo",
                      "value": round(last["samples_per_sec"], 1), "workers": args.workers,
                      "per_worker_batch": args.batch_size, "step_ms_p50": round(last["step_ms_p50"], 3),
                      "step_ms_p99": round(last["step_ms_p99"], 3), "epochs": rows}))


if __name__ == "__main__":
    main()
