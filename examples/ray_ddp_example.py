"""MNIST classifier trained data-parallel with ``RayAccelerator`` (optionally a
Tune sweep): the workflow of the reference's examples/ray_ddp_example.py on
this framework.  On MI355X workers each own one GPU; the MNIST MLP then runs
on the fused HIP step with the dataset resident in HBM, and gradients are
averaged by the native comm engine (xGMI one-shot allreduce / RCCL).

Data is synthetic MNIST-shaped (no network in this environment).

    python examples/ray_ddp_example.py --num-workers 2                 # CPU / gloo
    python examples/ray_ddp_example.py --num-workers 8 --use-gpu       # 8x MI355X
    python examples/ray_ddp_example.py --tune --num-samples 4 --num-workers 2 --use-gpu
    python examples/ray_ddp_example.py --smoke-test
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
from ray_lightning_accelerators_amd.models.mnist import MNISTClassifier  # noqa: E402
from ray_lightning_accelerators_amd.tune import TuneReportCallback  # noqa: E402


def train_mnist(config, data_dir=None, num_epochs=10, num_workers=1, use_gpu=False, callbacks=None):
    model = MNISTClassifier(config, data_dir)
    trainer = pl.Trainer(max_epochs=num_epochs, gpus=int(use_gpu), callbacks=list(callbacks or []),
                         accelerator=RayAccelerator(num_workers=num_workers, use_gpu=use_gpu))
    trainer.fit(model)
    return trainer


def tune_mnist(data_dir, num_samples=10, num_epochs=10, num_workers=1, use_gpu=False):
    config = {
        "layer_1": tune.choice([32, 64, 128]),
        "layer_2": tune.choice([64, 128, 256]),
        "lr": tune.loguniform(1e-4, 1e-1),
        "batch_size": tune.choice([32, 64, 128]),
    }
    reports = TuneReportCallback({"loss": "ptl/val_loss", "acc": "ptl/val_accuracy"}, on="validation_end")
    trainable = tune.with_parameters(train_mnist, data_dir=data_dir, num_epochs=num_epochs,
                                     num_workers=num_workers, use_gpu=use_gpu, callbacks=[reports])
    # the trial driver takes one CPU; its workers are reserved as "extra" resources
    analysis = tune.run(trainable, metric="loss", mode="min", config=config, num_samples=num_samples,
                        resources_per_trial={"cpu": 1, "gpu": 0, "extra_cpu": num_workers,
                                             "extra_gpu": num_workers * int(use_gpu)},
                        name="tune_mnist",
                        local_dir=os.environ.get("TUNE_RESULTS_DIR", os.path.join(tempfile.gettempdir(), "ray_results")))
    print("Best hyperparameters found were: ", analysis.best_config)
    return analysis


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-workers", type=int, default=1, help="Number of training workers to use.")
    ap.add_argument("--use-gpu", action="store_true", help="Use GPU for training.")
    ap.add_argument("--tune", action="store_true", help="Use Tune for hyperparameter tuning.")
    ap.add_argument("--num-samples", type=int, default=10, help="Number of samples to tune.")
    ap.add_argument("--num-epochs", type=int, default=10, help="Number of epochs to train for.")
    ap.add_argument("--smoke-test", action="store_true", help="Finish quickly for testing")
    ap.add_argument("--address", type=str, default=None, help="address of a running runtime head")
    args, _ = ap.parse_known_args(argv)

    num_epochs = 1 if args.smoke_test else args.num_epochs
    num_workers = 1 if args.smoke_test else args.num_workers
    use_gpu = False if args.smoke_test else args.use_gpu
    num_samples = 1 if args.smoke_test else args.num_samples
    if args.smoke_test:
        ray.init(num_cpus=2)
    else:
        ray.init(address=args.address)
    data_dir = os.path.join(tempfile.gettempdir(), "mnist_data_")
    try:
        if args.tune:
            tune_mnist(data_dir, num_samples, num_epochs, num_workers, use_gpu)
        else:
            config = {"layer_1": 32, "layer_2": 64, "lr": 1e-1, "batch_size": 32}
            train_mnist(config, data_dir, num_epochs, num_workers, use_gpu)
    finally:
        ray.shutdown()


if __name__ == "__main__":
    main()
