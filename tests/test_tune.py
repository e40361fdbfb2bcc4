"""Tune integration -- port of the reference's ray_lightning/tests/test_tune.py."""
import os

import pytest

from ray_lightning_accelerators_amd import HorovodRayAccelerator, RayAccelerator
from ray_lightning_accelerators_amd import runtime as ray
from ray_lightning_accelerators_amd import tune
from ray_lightning_accelerators_amd.tune import TuneReportCallback, TuneReportCheckpointCallback

from helpers import BoringModel, get_trainer


@pytest.fixture
def ray_start_4_cpus():
    info = ray.init(num_cpus=4, num_gpus=0)
    yield info
    ray.shutdown()


def train_func(dir, accelerator, use_gpu=False, callbacks=None):
    def _inner_train(config):
        model = BoringModel()
        trainer = get_trainer(dir, use_gpu=use_gpu, callbacks=callbacks, accelerator=accelerator, **config)
        trainer.fit(model)

    return _inner_train


def tune_test(dir, accelerator):
    callbacks = [TuneReportCallback(on="validation_end")]
    analysis = tune.run(train_func(dir, accelerator, callbacks=callbacks),
                        config={"max_epochs": tune.choice([1, 2, 3])},
                        resources_per_trial={"cpu": 0, "extra_cpu": 2}, num_samples=2,
                        local_dir=str(dir))
    assert all(analysis.results_df["training_iteration"] == analysis.results_df["config.max_epochs"])


def test_tune_iteration_ddp(tmpdir, ray_start_4_cpus):
    accelerator = RayAccelerator(num_workers=2, use_gpu=False)
    tune_test(tmpdir, accelerator)


def test_tune_iteration_horovod(tmpdir, ray_start_4_cpus):
    accelerator = HorovodRayAccelerator(num_hosts=1, num_slots=2, use_gpu=False)
    tune_test(tmpdir, accelerator)


def checkpoint_test(dir, accelerator):
    callbacks = [TuneReportCheckpointCallback(on="validation_end")]
    analysis = tune.run(train_func(dir, accelerator, callbacks=callbacks), config={"max_epochs": 2},
                        resources_per_trial={"cpu": 0, "extra_cpu": 2}, num_samples=1, local_dir=str(dir),
                        log_to_file=True, metric="val_loss", mode="min")
    assert analysis.best_checkpoint is not None
    assert os.path.exists(analysis.best_checkpoint)
    assert os.path.exists(os.path.join(analysis.best_checkpoint, "checkpoint"))


def test_checkpoint_ddp(tmpdir, ray_start_4_cpus):
    accelerator = RayAccelerator(num_workers=2, use_gpu=False)
    checkpoint_test(tmpdir, accelerator)


def test_checkpoint_horovod(tmpdir, ray_start_4_cpus):
    accelerator = HorovodRayAccelerator(num_hosts=1, num_slots=2, use_gpu=False)
    checkpoint_test(tmpdir, accelerator)


def test_report_metric_mapping(tmpdir, ray_start_4_cpus):
    """dict metrics map tune names -> Lightning names; best_config uses them."""
    callbacks = [TuneReportCallback({"loss": "val_loss"}, on="validation_end")]
    analysis = tune.run(train_func(tmpdir, RayAccelerator(num_workers=1), callbacks=callbacks),
                        config={"max_epochs": tune.grid_search([1, 2])}, resources_per_trial={"cpu": 0, "extra_cpu": 1},
                        num_samples=1, local_dir=str(tmpdir), metric="loss", mode="min")
    df = analysis.results_df
    assert len(df) == 2 and set(df["config.max_epochs"]) == {1, 2}
    assert "loss" in df.columns and (df["loss"] == 1.0).all()
    assert analysis.best_config["max_epochs"] in (1, 2)


def test_sample_space():
    cfgs = tune.sample.generate_variants(
        {"a": tune.choice([32, 64]), "lr": tune.loguniform(1e-4, 1e-1), "g": tune.grid_search([1, 2, 3])},
        num_samples=4, seed=0)
    assert len(cfgs) == 12
    assert all(c["a"] in (32, 64) and 1e-4 <= c["lr"] <= 1e-1 for c in cfgs)
    assert sorted({c["g"] for c in cfgs}) == [1, 2, 3]


class _GpuProbe:
    """Stands in for one RayAccelerator GPU worker: reports its pinned device and
    holds it for a moment, so concurrently running trials overlap."""

    def hold(self, seconds):
        import os
        import time

        t0 = time.time()
        time.sleep(seconds)
        return os.environ.get("HIP_VISIBLE_DEVICES"), t0, time.time()


def _packing_trainable(config):
    workers = [ray.remote(_GpuProbe).options(num_cpus=1, num_gpus=1).remote() for _ in range(2)]
    out = ray.get([w.hold.remote(6.0) for w in workers])  # > worst-case worker start skew
    for w in workers:
        ray.kill(w)
    tune.report(devices=",".join(d for d, _, _ in out), start=min(s for _, s, _ in out),
                end=max(e for _, _, e in out))


def test_tune_packs_4_trials_x_2_gpu_workers_on_8_gpus(tmpdir):
    """BASELINE config 4 topology: 4 trials x RayAccelerator(num_workers=2, use_gpu=True) on one
    8-GPU node (virtual GPU ledger: every device pinned to exactly one worker at a time)."""
    ray.init(num_cpus=16, num_gpus=0, _nodes=[{"ip": "127.0.0.1", "num_cpus": 16, "num_gpus": 8,
                                               "gpu_ids": [str(i) for i in range(8)]}])
    try:
        analysis = tune.run(_packing_trainable, config={"x": tune.choice([1, 2])}, num_samples=4,
                            resources_per_trial={"cpu": 1, "extra_cpu": 2, "extra_gpu": 2},
                            local_dir=str(tmpdir))
        df = analysis.results_df
        assert len(df) == 4
        devs = [d for s in df["devices"] for d in s.split(",")]
        assert sorted(devs) == [str(i) for i in range(8)], devs  # 8 distinct GPUs, one per worker
        starts, ends = list(df["start"]), list(df["end"])
        assert max(starts) < min(ends), "the 4 trials must run concurrently"
    finally:
        ray.shutdown()


def _report_once_and_return(config):
    tune.report(score=config["i"])


def test_last_report_of_a_finishing_trial_is_kept(tmpdir, ray_start_4_cpus):
    """A trial that reports once and returns at once: its report can still be in the
    queue when the runner sees the trial finish; it must land in the results, as must
    the first reports of other trials drained at that moment."""
    analysis = tune.run(_report_once_and_return, config={"i": tune.grid_search(list(range(8)))},
                        resources_per_trial={"cpu": 1}, local_dir=str(tmpdir))
    df = analysis.results_df
    assert len(df) == 8
    assert sorted(df["score"]) == list(range(8))


def _report_pid(config):
    import sys

    print("trial output", config["i"])  # goes to the trial's own stdout file (log_to_file)
    tune.report(pid=os.getpid(), cwd=os.getcwd(), redirected=sys.stdout is not sys.__stdout__)


def test_sequential_trials_recycle_the_trial_process(tmpdir, ray_start_4_cpus):
    """config.reuse_workers: a finished trial's process is parked and the next trial
    runs in it (no interpreter + torch start-up), with its own working directory and
    the previous trial's stdout redirection undone."""
    analysis = tune.run(_report_pid, config={"i": tune.grid_search(list(range(4)))},
                        resources_per_trial={"cpu": 1}, local_dir=str(tmpdir), max_concurrent_trials=1,
                        log_to_file=True)
    df = analysis.results_df
    assert len(df) == 4
    assert df["pid"].nunique() <= 2, list(df["pid"])  # trials after the first reuse its process
    for t in analysis.trials:
        assert t.last_result["cwd"] == t.logdir
        assert t.last_result["redirected"]
        with open(os.path.join(t.logdir, "stdout")) as f:
            assert f.read().count("trial output") == 1  # no other trial's output leaked in


def test_synthetic_mnist_pickles_by_spec_until_modified():
    """The dataset a model carries to its workers ships as its spec (not 47 MB of
    pixels) while untouched, and by value once changed."""
    import pickle

    from ray_lightning_accelerators_amd.models.data import SyntheticMNIST

    d = SyntheticMNIST(1000, seed=5)
    blob = pickle.dumps(d)
    assert len(blob) < 1024
    e = pickle.loads(blob)
    assert bool((e.images == d.images).all()) and bool((e.targets == d.targets).all())
    d.images[0, 0] = 3  # in place
    f = pickle.loads(pickle.dumps(d))
    assert int(f.images[0, 0]) == 3
    d2 = SyntheticMNIST(1000, seed=5)
    d2.targets = d2.targets.clone()  # replaced
    assert len(pickle.dumps(d2)) > 1024
