"""Single-process Trainer facade: PL 1.1 loop semantics and checkpoint format."""
import os

import pytest
import torch
from torch.utils.data import DataLoader

import ray_lightning_accelerators_amd.lightning as pl
from ray_lightning_accelerators_amd.lightning import Callback
from ray_lightning_accelerators_amd.lightning.callbacks import EarlyStopping, ModelCheckpoint
from ray_lightning_accelerators_amd.lightning.utilities import load_checkpoint
from ray_lightning_accelerators_amd.models.boring import BoringModel
from ray_lightning_accelerators_amd.models.data import RandomDataset
from ray_lightning_accelerators_amd.models.mnist import LightningMNISTClassifier


class HookRecorder(Callback):
    def __init__(self):
        self.calls = []

    def __getattribute__(self, name):
        if name.startswith("on_") or name in ("setup", "teardown"):
            rec = object.__getattribute__(self, "calls")

            def hook(trainer, pl_module, *a, **k):
                rec.append((name, trainer.running_sanity_check))
            return hook
        return object.__getattribute__(self, name)


def test_fit_returns_one_and_hook_order(tmpdir):
    rec = HookRecorder()
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=2, limit_train_batches=3, limit_val_batches=2,
                         callbacks=[rec])
    assert trainer.fit(BoringModel()) == 1
    names = [c[0] for c in rec.calls]
    assert names.index("on_sanity_check_start") < names.index("on_train_start")
    # validation (incl. on_validation_end) happens BEFORE on_epoch_end within an epoch
    first_epoch_end = names.index("on_epoch_end")
    assert "on_validation_end" in names[names.index("on_train_start"):first_epoch_end]
    sanity_val_end = [c for c in rec.calls if c[0] == "on_validation_end" and c[1]]
    assert len(sanity_val_end) == 1
    assert names.count("on_train_batch_end") == 6


def test_checkpoint_format_and_load(tmpdir):
    class HP(LightningMNISTClassifier):
        def __init__(self, config, data_dir=None):
            super().__init__(config, data_dir)
            self.save_hyperparameters()

    model = HP({"layer_1": 32, "layer_2": 32, "lr": 1e-3, "batch_size": 16})
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=4, limit_val_batches=2)
    trainer.fit(model)
    path = trainer.checkpoint_callback.best_model_path
    assert os.path.exists(path) and path.endswith(".ckpt")
    assert "lightning_logs/version_0/checkpoints" in path
    ckpt = load_checkpoint(path)
    for key in ("epoch", "global_step", "pytorch-lightning_version", "callbacks", "optimizer_states",
                "lr_schedulers", "state_dict", "hparams_name", "hyper_parameters"):
        assert key in ckpt, key
    assert set(ckpt["state_dict"]) == set(model.state_dict())
    st = ckpt["optimizer_states"][0]
    assert st["state"][0]["exp_avg"].shape == model.layer_1.weight.shape
    assert float(st["state"][0]["step"]) == 4
    assert "ModelCheckpoint" in ckpt["callbacks"]
    reloaded = HP.load_from_checkpoint(path)
    for k, v in model.state_dict().items():
        assert torch.allclose(reloaded.state_dict()[k], v)


def test_resume_from_checkpoint(tmpdir):
    t1 = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=2, limit_train_batches=2, limit_val_batches=1)
    t1.fit(BoringModel())
    path = t1.checkpoint_callback.best_model_path
    m2 = BoringModel()
    t2 = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, limit_train_batches=2, limit_val_batches=1,
                    resume_from_checkpoint=path)
    t2.fit(m2)
    assert t2.current_epoch == 2 or t2.current_epoch == 3


def test_lr_scheduler_steps_per_epoch(tmpdir):
    class M(BoringModel):
        def configure_optimizers(self):
            opt = torch.optim.SGD(self.parameters(), lr=1.0)
            return [opt], [torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)]

    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, limit_train_batches=2, limit_val_batches=1)
    trainer.fit(M())
    assert abs(trainer.optimizers[0].param_groups[0]["lr"] - 0.125) < 1e-9


def _train_weights(tmpdir, **kw):
    pl.seed_everything(3)
    model = BoringModel()
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, num_sanity_val_steps=0, logger=False,
                         checkpoint_callback=False, limit_val_batches=0, **kw)
    trainer.fit(model)
    return model.layer.weight.detach().clone()


def test_accumulate_grad_batches(tmpdir):
    class M(BoringModel):
        def __init__(self, bs):
            super().__init__()
            self.bs = bs

        def train_dataloader(self):
            return DataLoader(RandomDataset(32, 64, generator=torch.Generator().manual_seed(0)), batch_size=self.bs)

        def configure_optimizers(self):
            return torch.optim.SGD(self.parameters(), lr=0.1)

    def run(bs, acc):
        pl.seed_everything(3)
        m = M(bs)
        t = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, num_sanity_val_steps=0, logger=False,
                       checkpoint_callback=False, limit_val_batches=0, accumulate_grad_batches=acc)
        t.fit(m)
        return m.layer.weight.detach().clone(), t.global_step

    w_big, s_big = run(16, 1)
    w_acc, s_acc = run(8, 2)
    assert s_big == s_acc == 4
    assert torch.allclose(w_big, w_acc, atol=1e-6)


def test_fused_optimizer_matches_torch(tmpdir, monkeypatch):
    w_fused = _train_weights(tmpdir)
    monkeypatch.setenv("RLA_FUSED_OPTIM", "0")
    w_torch = _train_weights(tmpdir)
    assert torch.allclose(w_fused, w_torch, atol=1e-6)


def test_gradient_clipping_runs(tmpdir):
    w = _train_weights(tmpdir, gradient_clip_val=1e-3)
    w_free = _train_weights(tmpdir)
    assert not torch.allclose(w, w_free)


def test_early_stopping_state_in_checkpoint(tmpdir):
    es = EarlyStopping(monitor="val_loss", patience=1)
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=10, limit_train_batches=2, limit_val_batches=2,
                         callbacks=[es])
    trainer.fit(BoringModel())
    assert trainer.current_epoch == 1  # epoch 0 best, epoch 1 no improvement -> stop
    ckpt = trainer.checkpoint_connector.dump_checkpoint()
    assert ckpt["callbacks"]["EarlyStopping"]["patience"] == 1


def test_logged_metrics_reach_callback_metrics(tmpdir):
    model = LightningMNISTClassifier({"layer_1": 32, "layer_2": 64, "lr": 1e-3, "batch_size": 32})
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=5, limit_val_batches=3)
    trainer.fit(model)
    for k in ("ptl/train_loss", "ptl/train_accuracy", "ptl/val_loss", "ptl/val_accuracy"):
        assert k in trainer.callback_metrics, k
    assert os.path.exists(os.path.join(trainer.log_dir, "metrics.csv"))


def test_test_loop_returns_results(tmpdir):
    class M(BoringModel):
        def test_step(self, batch, batch_idx):
            out = super().test_step(batch, batch_idx)
            self.log("test_loss", out["y"])
            return out

    model = M()
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=2, limit_val_batches=1,
                         limit_test_batches=3)
    trainer.fit(model)
    res = trainer.test(model)
    assert isinstance(res, list) and "test_loss" in res[0]


def test_model_checkpoint_monitor_explicit(tmpdir):
    class M(BoringModel):
        def validation_step(self, batch, batch_idx):
            self.log("score", torch.tensor(float(self.current_epoch)))
            return super().validation_step(batch, batch_idx)

    mc = ModelCheckpoint(monitor="score", mode="max")
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, limit_train_batches=1, limit_val_batches=1,
                         callbacks=[mc])
    trainer.fit(M())
    assert "epoch=2" in os.path.basename(mc.best_model_path)
    assert float(mc.best_model_score) == 2.0


def test_new_best_checkpoint_names_itself_and_resume_keeps_score(tmpdir):
    """PL 1.1.7 _update_best_and_save: the best / current fields are set BEFORE the
    dump, so a new-best file's callbacks[ModelCheckpoint] names that file and its
    score (reference tune.py:138 ships this dict; tests/utils.py:129-134 reloads it);
    resuming from it restores the best score and path."""
    class M(BoringModel):
        def validation_step(self, batch, batch_idx):
            self.log("score", torch.tensor(float(self.current_epoch) + 0.5))
            return super().validation_step(batch, batch_idx)

    mc = ModelCheckpoint(dirpath=str(tmpdir), monitor="score", mode="max", save_last=True)
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, limit_train_batches=1, limit_val_batches=1,
                         callbacks=[mc])
    trainer.fit(M())
    trainer.wait_checkpoints()
    best = mc.best_model_path
    ck = load_checkpoint(best)["callbacks"]["ModelCheckpoint"]
    assert ck["best_model_path"] == best
    assert float(ck["best_model_score"]) == 2.5 and float(ck["current_score"]) == 2.5
    last = load_checkpoint(os.path.join(str(tmpdir), "last.ckpt"))["callbacks"]["ModelCheckpoint"]
    assert last["best_model_path"] == best
    # resume: the restored callback keeps the best score / path of the file
    mc2 = ModelCheckpoint(dirpath=str(tmpdir), monitor="score", mode="max")
    t2 = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, limit_train_batches=1, limit_val_batches=1,
                    callbacks=[mc2], resume_from_checkpoint=best)
    t2.fit(M())
    assert float(mc2.best_model_score) == 2.5 and mc2.best_model_path == best


def test_model_checkpoint_without_monitor_names_itself(tmpdir):
    mc = ModelCheckpoint(dirpath=str(tmpdir))
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=2, limit_train_batches=1, limit_val_batches=0,
                         callbacks=[mc], logger=False)
    trainer.fit(BoringModel())
    trainer.wait_checkpoints()
    ck = load_checkpoint(mc.best_model_path)["callbacks"]["ModelCheckpoint"]
    assert ck["best_model_path"] == mc.best_model_path


def test_async_checkpoint_writes_land_before_fit_returns(tmpdir, monkeypatch):
    """RLAConfig.async_checkpoint: ModelCheckpoint's writes (and its top-k removals)
    run on the background writer, in order; every file is complete when fit returns."""
    from ray_lightning_accelerators_amd.config import set_config
    from ray_lightning_accelerators_amd.lightning.utilities import load_checkpoint

    class M(BoringModel):
        def validation_step(self, batch, batch_idx):
            self.log("score", torch.tensor(float(self.current_epoch)))
            return super().validation_step(batch, batch_idx)

    monkeypatch.setenv("RLA_ASYNC_CHECKPOINT", "1")
    set_config(None)
    try:
        mc = ModelCheckpoint(monitor="score", mode="max")
        trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, limit_train_batches=2, limit_val_batches=1,
                             callbacks=[mc])
        trainer.fit(M())
        assert trainer._ckpt_writer is not None  # the background path ran
        assert "epoch=2" in os.path.basename(mc.best_model_path)
        ckpts = [f for f in os.listdir(os.path.dirname(mc.best_model_path)) if f.endswith(".ckpt")]
        assert ckpts == [os.path.basename(mc.best_model_path)]  # earlier bests removed after their writes
        ck = load_checkpoint(mc.best_model_path)
        # PL 1.1 layout: epoch and global_step are stored + 1
        assert ck["epoch"] == 3 and ck["global_step"] == trainer.global_step + 1 and ck["state_dict"]
    finally:
        set_config(None)


@pytest.mark.parametrize("bad", [None])
def test_seed_everything_env(bad):
    s = pl.seed_everything(42)
    assert s == 42 and os.environ["PL_GLOBAL_SEED"] == "42"


def test_owner_state_consolidated_at_validation_end_not_in_dump(tmpdir):
    """under the owner exchange protocol the Adam-state consolidation is a
    collective.  It runs on EVERY rank at validation end (before ModelCheckpoint,
    whose per-rank save decision may differ); the dump itself then skips it."""
    class FakeFused:
        calls = 0

        def sync_optimizer_state(self):
            FakeFused.calls += 1

    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, callbacks=[ModelCheckpoint()])
    trainer._fused = FakeFused()
    trainer.world_size = 2
    trainer.training = True
    trainer.global_step = 7
    opt = torch.optim.Adam([torch.nn.Parameter(torch.zeros(2))])
    trainer._consolidate_optimizer_state()
    assert FakeFused.calls == 1
    trainer._optimizer_state_dict(opt)
    assert FakeFused.calls == 1, "dump re-ran the collective at the consolidated step"
    trainer.global_step = 8
    trainer._optimizer_state_dict(opt)
    assert FakeFused.calls == 2


def test_owner_state_consolidated_before_every_save_without_validation(tmpdir, monkeypatch):
    """with no validation loop the checkpoint callbacks save at every
    training-epoch end and at train end.  The owner-protocol consolidation (a
    collective) must run on every rank BEFORE each of those save points, never only
    inside rank 0's dump."""
    events = []
    real = pl.Trainer._consolidate_optimizer_state

    def consolidate(self):
        events.append(("consolidate", self.global_step))
        real(self)

    monkeypatch.setattr(pl.Trainer, "_consolidate_optimizer_state", consolidate)

    class Ck(ModelCheckpoint):
        def on_validation_end(self, trainer, pl_module):
            events.append(("save", trainer.global_step))
            super().on_validation_end(trainer, pl_module)

        def on_train_end(self, trainer, pl_module):
            events.append(("train_end", trainer.global_step))
            super().on_train_end(trainer, pl_module)

    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=2, limit_train_batches=2, limit_val_batches=0,
                         callbacks=[Ck(dirpath=str(tmpdir))])
    trainer.fit(BoringModel())
    saves = [i for i, e in enumerate(events) if e[0] in ("save", "train_end")]
    assert len(saves) == 3, events
    for i in saves:
        assert i > 0 and events[i - 1] == ("consolidate", events[i][1]), events
