"""Failure detection + teardown and profiling hooks (§5.1).

The reference is fail-fast (util.py:102-103 re-raises the first worker
exception) but leaks its actors on that path; here an injected worker fault
must reach the driver naming the rank, and every worker actor must be dead
afterwards.  A worker that vanishes without a Python exception (os._exit)
must be detected as well.
"""
import pytest
import torch

import ray_lightning_accelerators_amd.runtime as ray
from ray_lightning_accelerators_amd import HorovodRayAccelerator, RayAccelerator
from ray_lightning_accelerators_amd import lightning as pl
from ray_lightning_accelerators_amd.models.boring import BoringModel
from ray_lightning_accelerators_amd.utils.profiling import SimpleProfiler, StepTimer, resolve_profiler


@pytest.fixture
def ray_4_cpus():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _alive_workers():
    return [a for a in ray.actors().values() if a.get("State") == ray.ALIVE and "Queue" not in a.get("ClassName", "")]


@pytest.mark.parametrize("kind", ["raise", "exit"])
def test_ddp_worker_fault_surfaces_and_tears_down(tmpdir, ray_4_cpus, monkeypatch, kind):
    monkeypatch.setenv("RLA_FAULT_RANK", "1")
    monkeypatch.setenv("RLA_FAULT_STEP", "2")
    monkeypatch.setenv("RLA_FAULT_KIND", kind)
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=6, limit_val_batches=2,
                         accelerator=RayAccelerator(num_workers=2))
    with pytest.raises(Exception) as ei:
        trainer.fit(BoringModel())
    msg = str(ei.value)
    if kind == "raise":
        assert "injected fault on rank 1 at step 2" in msg
    assert not _alive_workers()


def test_horovod_worker_fault_surfaces(tmpdir, ray_4_cpus, monkeypatch):
    monkeypatch.setenv("RLA_FAULT_RANK", "0")
    monkeypatch.setenv("RLA_FAULT_STEP", "1")
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=4, limit_val_batches=2,
                         accelerator=HorovodRayAccelerator(num_slots=2))
    with pytest.raises(Exception) as ei:
        trainer.fit(BoringModel())
    assert "injected fault on rank 0 at step 1" in str(ei.value)


def test_simple_profiler_reports_training_batches(tmpdir):
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=5, limit_val_batches=1,
                         profiler="simple")
    assert trainer.fit(BoringModel()) == 1
    st = trainer.profiler.stats()
    assert st["run_training_batch"]["calls"] == 5
    assert "run_training_batch" in trainer.profiler_summary


def test_profiler_resolution():
    assert isinstance(resolve_profiler(True), SimpleProfiler)
    assert resolve_profiler("gpu").cuda_sync == torch.cuda.is_available()
    with pytest.raises(ValueError):
        resolve_profiler("nope")
    assert StepTimer().summary() == {}


def test_trainer_surfaces_collective_error(tmpdir, monkeypatch):
    """A timed-out xGMI poll / RCCL async error recorded by the native communicator
    is raised at the end of the epoch (fail-fast), not silently trained through."""
    import pytest

    import ray_lightning_accelerators_amd.lightning as pl
    from ray_lightning_accelerators_amd.models.boring import BoringModel
    from ray_lightning_accelerators_amd.parallel import comm as comm_mod

    class _BadComm:
        def check(self):
            raise RuntimeError("collective failure on rank 0: xGMI allreduce: peer flag poll timed out")

    monkeypatch.setattr(comm_mod, "get_native_comm", lambda create=True, **kw: _BadComm())
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=2, limit_val_batches=1,
                         checkpoint_callback=False)
    with pytest.raises(RuntimeError, match="peer flag poll timed out"):
        trainer.fit(BoringModel())
