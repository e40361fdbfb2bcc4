"""RayAccelerator on CPU / gloo -- port of the reference's ray_lightning/tests/test_ddp.py."""
import time

import pytest
from torch.utils.data import DistributedSampler

import ray_lightning_accelerators_amd.lightning as pl
from ray_lightning_accelerators_amd import RayAccelerator
from ray_lightning_accelerators_amd import runtime as ray
from ray_lightning_accelerators_amd.lightning import Callback
from ray_lightning_accelerators_amd.lightning.callbacks import EarlyStopping
from ray_lightning_accelerators_amd.models.datamodules import MNISTDataModule
from ray_lightning_accelerators_amd.models.mnist import LightningMNISTClassifier

from helpers import BoringModel, get_trainer, load_test, predict_test, train_test


@pytest.fixture
def ray_start_2_cpus():
    info = ray.init(num_cpus=2, num_gpus=0)
    yield info
    ray.shutdown()


@pytest.fixture
def seed():
    pl.seed_everything(0)


@pytest.mark.parametrize("num_workers", [1, 2])
def test_actor_creation(tmpdir, ray_start_2_cpus, num_workers):
    """N live actors during training; all DEAD after fit (reference test_ddp.py:29-42)."""
    model = BoringModel()

    def check_num_actor():
        assert len(ray.actors()) == num_workers

    model.on_epoch_end = check_num_actor
    accelerator = RayAccelerator(num_workers=num_workers)
    trainer = get_trainer(tmpdir, accelerator=accelerator)
    trainer.fit(model)
    assert all(actor["State"] == ray.gcs_utils.ActorTableData.DEAD for actor in ray.actors().values())


def test_distributed_sampler(tmpdir, ray_start_2_cpus):
    model = BoringModel()
    assert not isinstance(model.train_dataloader().sampler, DistributedSampler)

    class DistributedSamplerCallback(Callback):
        def on_train_start(self, trainer, pl_module):
            s = trainer.train_dataloader.sampler
            assert isinstance(s, DistributedSampler)
            assert s.shuffle
            assert s.num_replicas == 2
            assert s.rank == trainer.global_rank

        def on_validation_start(self, trainer, pl_module):
            s = trainer.val_dataloaders[0].sampler
            assert isinstance(s, DistributedSampler)
            assert not s.shuffle
            assert s.num_replicas == 2
            assert s.rank == trainer.global_rank

        def on_test_start(self, trainer, pl_module):
            s = trainer.test_dataloaders[0].sampler
            assert isinstance(s, DistributedSampler)
            assert not s.shuffle
            assert s.num_replicas == 2
            assert s.rank == trainer.global_rank

    accelerator = RayAccelerator(num_workers=2)
    trainer = get_trainer(tmpdir, accelerator=accelerator, callbacks=[DistributedSamplerCallback()])
    trainer.fit(model)
    trainer.test(model)


@pytest.mark.parametrize("num_workers", [1, 2])
def test_train(tmpdir, ray_start_2_cpus, num_workers):
    model = BoringModel()
    accelerator = RayAccelerator(num_workers=num_workers)
    trainer = get_trainer(tmpdir, accelerator=accelerator)
    train_test(trainer, model)


@pytest.mark.parametrize("num_workers", [1, 2])
def test_load(tmpdir, ray_start_2_cpus, num_workers):
    model = BoringModel()
    accelerator = RayAccelerator(num_workers=num_workers, use_gpu=False)
    trainer = get_trainer(tmpdir, accelerator=accelerator)
    load_test(trainer, model)


@pytest.mark.parametrize("num_workers", [1, 2])
def test_predict(tmpdir, ray_start_2_cpus, seed, num_workers):
    config = {"layer_1": 32, "layer_2": 32, "lr": 1e-2, "batch_size": 32}
    model = LightningMNISTClassifier(config, tmpdir)
    dm = MNISTDataModule(data_dir=tmpdir, num_workers=1, batch_size=config["batch_size"])
    accelerator = RayAccelerator(num_workers=num_workers, use_gpu=False)
    trainer = get_trainer(tmpdir, limit_train_batches=10, max_epochs=1, accelerator=accelerator)
    predict_test(trainer, model, dm)


def test_early_stop(tmpdir, ray_start_2_cpus):
    """Constant val loss + patience 2: best checkpoint has val_epoch == 2 (sanity + epoch 0)."""
    model = BoringModel()
    accelerator = RayAccelerator(num_workers=1, use_gpu=False)
    early_stop = EarlyStopping(monitor="val_loss", patience=2, verbose=True)
    trainer = get_trainer(tmpdir, max_epochs=500, accelerator=accelerator, callbacks=[early_stop],
                          limit_train_batches=1.0, limit_val_batches=1.0, progress_bar_refresh_rate=1)
    trainer.fit(model)
    trained_model = BoringModel.load_from_checkpoint(trainer.checkpoint_callback.best_model_path)
    assert trained_model.val_epoch == 2, trained_model.val_epoch


def test_seed_and_cpus_per_worker_alias(tmpdir, ray_start_2_cpus):
    """README spelling ``cpus_per_worker`` is accepted; PL_GLOBAL_SEED reaches the workers."""
    import os

    pl.seed_everything(1234)
    seen = []

    class SeedCheck(Callback):
        def on_train_start(self, trainer, pl_module):
            assert os.environ.get("PL_GLOBAL_SEED") == "1234"

    acc = RayAccelerator(num_workers=2, cpus_per_worker=1)
    assert acc.num_cpus_per_worker == 1
    trainer = get_trainer(tmpdir, accelerator=acc, callbacks=[SeedCheck()])
    assert trainer.fit(BoringModel()) == 1
    del seen


def test_worker_failure_tears_down(tmpdir, ray_start_2_cpus):
    """A worker exception surfaces on the driver and the actors are still torn down."""

    class Boom(BoringModel):
        def training_step(self, batch, batch_idx):
            if self.global_rank == 1 and batch_idx == 2:
                raise RuntimeError("injected failure")
            return super().training_step(batch, batch_idx)

    acc = RayAccelerator(num_workers=2)
    trainer = get_trainer(tmpdir, accelerator=acc)
    with pytest.raises(RuntimeError, match="injected failure"):
        trainer.fit(Boom())
    import time

    time.sleep(0.5)
    assert all(a["State"] == "DEAD" for a in ray.actors().values())


def test_recycled_worker_pair_across_two_fits(tmpdir, monkeypatch):
    """A world-2 worker pair is parked after one fit and taken over by the next
    (the Tune config-4 pattern: trials of RayAccelerator(num_workers=2) back to
    back).  The second fit must find a FRESH process group (new rendezvous, the
    first's destroyed in __rla_park__), a fresh session and config, and train
    correctly -- in the SAME processes (gloo stand-in for the
    GPU path, RLA_REUSE_CPU_WORKERS)."""
    import os

    import torch
    import torch.distributed as dist

    from ray_lightning_accelerators_amd.config import set_config

    monkeypatch.setenv("RLA_REUSE_CPU_WORKERS", "1")
    set_config(None)

    class PidModel(BoringModel):
        def __init__(self):
            super().__init__()
            self.register_buffer("pids", torch.zeros(2, dtype=torch.int64))
            self.register_buffer("groups", torch.zeros(1, dtype=torch.int64))

        def on_train_start(self):
            # both ranks' pids reach rank 0 (whose state dict comes back) through the
            # process group this fit created
            t = torch.zeros(2, dtype=torch.int64)
            t[dist.get_rank()] = os.getpid()
            dist.all_reduce(t)
            self.pids.copy_(t)
            self.groups.fill_(dist.get_world_size())

    ray.init(num_cpus=4, num_gpus=0)
    try:
        seen = []
        for fit in range(2):
            model = PidModel()
            trainer = get_trainer(tmpdir, accelerator=RayAccelerator(num_workers=2))
            train_test(trainer, model)
            assert int(model.groups) == 2
            seen.append(sorted(int(p) for p in model.pids))
            time.sleep(0.5)  # the park acknowledgement (the next create waits for it anyway)
        assert seen[0] == seen[1] and 0 not in seen[0], seen
    finally:
        ray.shutdown()
        set_config(None)
