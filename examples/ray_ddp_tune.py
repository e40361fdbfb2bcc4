"""Tune sweep over the MNIST classifier, each trial a multi-worker
``RayAccelerator`` job fed by a ``LightningDataModule`` (the workflow of the
reference's examples/ray_ddp_tune.py).

Packing on one 8x MI355X node: trial drivers reserve no GPU (``"gpu": 0``);
each trial's workers reserve ``extra_gpu = num_workers``, so 4 trials x 2
workers fill the 8 GPUs concurrently (BASELINE.json config 4).  Every trial
reports ``loss``/``acc`` at each validation end and checkpoints with
``TuneReportCheckpointCallback`` (Lightning checkpoint format).

    python examples/ray_ddp_tune.py --num-samples 4 --num-workers 2 --use-gpu
    python examples/ray_ddp_tune.py --smoke-test
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ray_lightning_accelerators_amd.runtime as ray  # noqa: E402
from ray_lightning_accelerators_amd import RayAccelerator  # noqa: E402
from ray_lightning_accelerators_amd import lightning as pl  # noqa: E402
from ray_lightning_accelerators_amd import tune  # noqa: E402
from ray_lightning_accelerators_amd.models.datamodules import MNISTDataModule  # noqa: E402
from ray_lightning_accelerators_amd.models.mnist import LightningMNISTClassifier  # noqa: E402
from ray_lightning_accelerators_amd.tune import TuneReportCheckpointCallback  # noqa: E402


def train_mnist(config, data_dir=None, num_epochs=10, num_workers=1, use_gpu=False, callbacks=None):
    def prepare_on_worker():
        # each worker materialises the dataset once (the reference downloads MNIST here)
        MNISTDataModule(data_dir=data_dir).prepare_data()

    model = LightningMNISTClassifier(config, data_dir)
    trainer = pl.Trainer(max_epochs=num_epochs, gpus=int(use_gpu), callbacks=list(callbacks or []),
                         progress_bar_refresh_rate=0,
                         accelerator=RayAccelerator(num_workers=num_workers, use_gpu=use_gpu,
                                                    init_hook=prepare_on_worker))
    dm = MNISTDataModule(data_dir=data_dir, num_workers=1, batch_size=config["batch_size"])
    trainer.fit(model, dm)


def tune_mnist(data_dir, num_samples=10, num_epochs=10, num_workers=1, use_gpu=False):
    config = {
        "layer_1": tune.choice([32, 64, 128]),
        "layer_2": tune.choice([64, 128, 256]),
        "lr": tune.loguniform(1e-4, 1e-1),
        "batch_size": tune.choice([32, 64, 128]),
    }
    callbacks = [TuneReportCheckpointCallback({"loss": "ptl/val_loss", "acc": "ptl/val_accuracy"},
                                              filename="checkpoint", on="validation_end")]
    trainable = tune.with_parameters(train_mnist, data_dir=data_dir, num_epochs=num_epochs,
                                     num_workers=num_workers, use_gpu=use_gpu, callbacks=callbacks)
    analysis = tune.run(trainable, metric="loss", mode="min", config=config, num_samples=num_samples,
                        resources_per_trial={"cpu": 1, "gpu": 0, "extra_cpu": num_workers,
                                             "extra_gpu": num_workers * int(use_gpu)},
                        name="tune_mnist",
                        local_dir=os.environ.get("TUNE_RESULTS_DIR", os.path.join(tempfile.gettempdir(), "ray_results")))
    print("Best hyperparameters found were: ", analysis.best_config)
    print("Best checkpoint: ", analysis.best_checkpoint)
    return analysis


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-workers", type=int, default=1, help="Number of training workers to use.")
    ap.add_argument("--use-gpu", action="store_true", help="Use GPU for training.")
    ap.add_argument("--num-samples", type=int, default=10, help="Number of samples to tune.")
    ap.add_argument("--num-epochs", type=int, default=10, help="Number of epochs to train for.")
    ap.add_argument("--smoke-test", action="store_true", help="Finish quickly for testing")
    ap.add_argument("--address", type=str, default=None, help="address of a running runtime head")
    args, _ = ap.parse_known_args(argv)
    num_epochs = 1 if args.smoke_test else args.num_epochs
    num_samples = 1 if args.smoke_test else args.num_samples
    if args.smoke_test:
        ray.init(num_cpus=3)
    else:
        ray.init(address=args.address)
    data_dir = os.path.join(tempfile.gettempdir(), "mnist_data_")
    try:
        return tune_mnist(data_dir, num_samples, num_epochs, args.num_workers, args.use_gpu)
    finally:
        ray.shutdown()


if __name__ == "__main__":
    main()
