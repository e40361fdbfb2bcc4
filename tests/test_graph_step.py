"""Trainer-level graph-captured autograd step (lightning/graph_step.py).

CPU: the step body runs eagerly through the same path a capture records (device
ring for the logged values, resident-data gather, device step / LR scalars of the
fused optimizer) and must train bit-identically to the plain eager Trainer; a
training_step that reads device values on the host falls back cleanly.
GPU: the captured replays match the eager Trainer, ResNet-50 runs captured."""
import os

import pytest
import torch
import torch.nn.functional as F
from torch import nn
from torch.utils.data import DataLoader, TensorDataset

import ray_lightning_accelerators_amd.lightning as pl
from ray_lightning_accelerators_amd.lightning.graph_step import GraphedTrainStep, HostReadProbe
from ray_lightning_accelerators_amd.lightning.sampling import gather_rows, resident_tensors


class Tiny(pl.LightningModule):
    """Conv + linear classifier: BN running stats, SGD-momentum, a logged metric."""

    hip_graph_step = True

    def __init__(self, n=96, batch=8, opt="sgd", sched=False, log_acc=True):
        super().__init__()
        torch.manual_seed(0)
        g = torch.Generator().manual_seed(0)
        self.x = torch.randn(n, 3, 8, 8, generator=g)
        self.y = torch.randint(0, 5, (n,), generator=g)
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.bn = nn.BatchNorm2d(8)
        self.fc = nn.Linear(8, 5)
        self.batch, self.opt_kind, self.sched, self.log_acc = batch, opt, sched, log_acc

    def forward(self, x):
        h = F.relu(self.bn(self.conv(x)))
        return self.fc(h.mean((2, 3)))

    def training_step(self, batch, batch_idx):
        x, y = batch
        logits = self(x)
        loss = F.cross_entropy(logits, y)
        self.log("train_loss", loss)
        if self.log_acc:
            self.log("train_acc", (logits.argmax(1) == y).float().mean())
        return loss

    def configure_optimizers(self):
        if self.opt_kind == "adam":
            opt = torch.optim.Adam(self.parameters(), lr=1e-2)
        else:
            opt = torch.optim.SGD(self.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        if self.sched:
            return [opt], [{"scheduler": torch.optim.lr_scheduler.StepLR(opt, 2, 0.5), "interval": "step"}]
        return opt

    def train_dataloader(self):
        return DataLoader(TensorDataset(self.x, self.y), batch_size=self.batch, shuffle=True, drop_last=True)


class HostSync(Tiny):
    def training_step(self, batch, batch_idx):
        loss = super().training_step(batch, batch_idx)
        if loss.item() > 1e9:  # a host read of a device value: not replayable
            print("huge")
        return loss


class Recorder(pl.Callback):
    def __init__(self):
        self.losses = []

    def on_train_epoch_end(self, trainer, pl_module, outputs=None):
        self.losses.extend(float(o["loss"]) for o in outputs)


def _fit(model, tmpdir, name, epochs=2, **kw):
    rec = Recorder()
    t = pl.Trainer(default_root_dir=os.path.join(str(tmpdir), name), max_epochs=epochs, callbacks=[rec],
                   progress_bar_refresh_rate=0, log_every_n_steps=3, **kw)
    torch.manual_seed(1)
    assert t.fit(model) == 1
    return t, rec


@pytest.mark.parametrize("opt,sched", [("sgd", False), ("adam", False), ("sgd", True)])
def test_graph_body_matches_eager_trainer(tmpdir, opt, sched):
    t_g, r_g = _fit(Tiny(opt=opt, sched=sched), tmpdir, "g")
    m_e = Tiny(opt=opt, sched=sched)
    m_e.hip_graph_step = False
    t_e, r_e = _fit(m_e, tmpdir, "e")
    assert isinstance(t_g._fused, GraphedTrainStep) and t_e._fused is None
    assert not t_g._fused.failed and t_g._fused.steps_done == 24
    assert r_g.losses == r_e.losses and len(r_g.losses) == 24
    for (k, a), b in zip(t_g.model.state_dict().items(), t_e.model.state_dict().values()):
        assert torch.equal(a, b), k
    assert t_g.global_step == t_e.global_step == 24
    assert float(t_g.callback_metrics["train_acc"]) == float(t_e.callback_metrics["train_acc"])
    # optimizer state (checkpoint format) identical, Adam's per-parameter step included
    sd_g, sd_e = t_g.optimizers[0].state_dict(), t_e.optimizers[0].state_dict()
    for i in sd_e["state"]:
        for k, v in sd_e["state"][i].items():
            assert torch.equal(sd_g["state"][i][k], v), (i, k)
    # the logger rows (every log_every_n_steps) are the same values
    rows = lambda t: open(os.path.join(t.logger.log_dir, "metrics.csv")).read()  # noqa: E731
    assert rows(t_g) == rows(t_e)


def test_resident_dataset_path(tmpdir):
    """TensorDataset batches are gathered from resident columns with the sampler's
    order (many steps per dispatch), identical to iterating the loader."""
    t_g, r_g = _fit(Tiny(), tmpdir, "g", epochs=3)
    f = t_g._fused
    assert f._resident is not None and f.describe()["resident_data"]
    m_e = Tiny()
    m_e.hip_graph_step = False
    t_e, r_e = _fit(m_e, tmpdir, "e", epochs=3)
    assert r_g.losses == r_e.losses


def test_host_read_falls_back(tmpdir):
    t_h, r_h = _fit(HostSync(), tmpdir, "h")
    f = t_h._fused
    assert f.failed and "item" in f.reason and "test_graph_step.py" in f.reason
    m_e = Tiny()
    m_e.hip_graph_step = False
    t_e, r_e = _fit(m_e, tmpdir, "e")
    assert r_h.losses == r_e.losses  # the fallback trains exactly like eager


class LogsFloat(Tiny):
    """self.log of a Python float: rejected by the step body (after the forward) --
    on the RESIDENT path too, where the batch is a device-gathered sentinel."""

    def training_step(self, batch, batch_idx):
        loss = super().training_step(batch, batch_idx)
        self.log("lr_host", 0.05)
        return loss


def test_resident_rejection_falls_back_like_eager(tmpdir):
    """a step rejected on the resident-data path must not crash the fit:
    the gathered batch is re-run by the eager path, every later step too, and the
    forward of the rejected attempt leaves no trace (BN running statistics and
    num_batches_tracked updated once) -- bit-identical to the plain eager Trainer."""
    t_f, r_f = _fit(LogsFloat(), tmpdir, "f", epochs=2)
    f = t_f._fused
    assert f.failed and "lr_host" in f.reason
    m_e = LogsFloat()
    m_e.hip_graph_step = False
    t_e, r_e = _fit(m_e, tmpdir, "e", epochs=2)
    assert r_f.losses == r_e.losses and len(r_f.losses) == 24
    assert t_f.global_step == t_e.global_step == 24
    for (k, a), b in zip(t_f.model.state_dict().items(), t_e.model.state_dict().values()):
        assert torch.equal(a, b), k


def test_static_rejections(tmpdir):
    class Hooked(Tiny):
        def on_after_backward(self):
            pass

    t, _ = _fit(Hooked(), tmpdir, "a", epochs=1)
    assert t._fused is None and "on_after_backward" in t._graph_step_reason
    t, _ = _fit(Tiny(), tmpdir, "b", epochs=1, accumulate_grad_batches=2)
    assert t._fused is None and "accumulate" in t._graph_step_reason


def test_host_read_probe_attribution():
    probe = HostReadProbe()
    x = torch.ones(3)
    with probe:
        y = x * 2
        float(y.sum())
        y.tolist()
        _ = y + 1
    assert len(probe.reads) == 2 and all("test_graph_step.py" in r for r in probe.reads)


def test_gather_rows_keeps_channels_last():
    x = torch.randn(10, 3, 4, 4).contiguous(memory_format=torch.channels_last)
    idx = torch.tensor([3, 1, 7])
    g = gather_rows(x, idx)
    assert g.is_contiguous(memory_format=torch.channels_last) and torch.equal(g, x[idx])


def test_synthetic_imagenet_resident_matches_items():
    from torch.utils.data import Subset

    from ray_lightning_accelerators_amd.models.resnet import SyntheticImageNet

    ds = SyntheticImageNet(20, 16, 7, seed=3)
    cols, idx_map = resident_tensors(Subset(ds, [4, 2, 9]), torch.device("cpu"))
    assert idx_map.tolist() == [4, 2, 9]
    x, y = cols
    for i in (0, 9, 19):
        a, b = ds[i]
        assert torch.equal(x[i], a) and int(y[i]) == b


def test_epoch_checkpoint_without_validation(tmpdir):
    """PL 1.1: with no validation loop the checkpoint callbacks run at every
    training-epoch end (TrainLoop.check_checkpoint_callback)."""
    saved = []

    class CK(pl.callbacks.ModelCheckpoint):
        def save_checkpoint(self, trainer, pl_module):
            saved.append(trainer.global_step)
            return super().save_checkpoint(trainer, pl_module)

    m = Tiny()
    m.hip_graph_step = False
    t = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=3, callbacks=[CK()], progress_bar_refresh_rate=0)
    t.fit(m)
    assert saved[:3] == [12, 24, 36]
    assert os.path.exists(t.checkpoint_callback.best_model_path)


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [True, False])
def test_gpu_captured_matches_eager(tmpdir, resident):
    """Captured replays (after the warm-up) train like the eager Trainer."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")

    class G(Tiny):
        def train_dataloader(self):
            dl = super().train_dataloader()
            if resident:
                return dl

            class Plain(torch.utils.data.Dataset):  # not resident-capable: loader + static buffers
                def __init__(s, ds):
                    s.ds = ds

                def __len__(s):
                    return len(s.ds)

                def __getitem__(s, i):
                    return s.ds[i]

            return DataLoader(Plain(dl.dataset), batch_size=self.batch, shuffle=True, drop_last=True)

    t_g, r_g = _fit(G(), tmpdir, "g", gpus=1)
    f = t_g._fused
    assert f.graph is not None and f.replays == 24 - f.warmup, f.describe()
    assert (f._resident is not None) == resident
    m_e = G()
    m_e.hip_graph_step = False
    t_e, r_e = _fit(m_e, tmpdir, "e", gpus=1)
    torch.testing.assert_close(torch.tensor(r_g.losses), torch.tensor(r_e.losses), rtol=1e-4, atol=1e-5)
    for (k, a), b in zip(t_g.model.state_dict().items(), t_e.model.state_dict().values()):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-4, atol=1e-5, msg=k)


class _Dist(Tiny):
    """Tiny, picklable across the runtime's actors (module-level class)."""


class _AssertGraphStep(pl.Callback):
    """Worker side: the graph step ran its body (no fallback); Horovod's reduction
    was adopted by the GradSynchronizer."""

    def __init__(self, want, horovod):
        self.want, self.horovod = want, horovod

    def on_train_end(self, trainer, pl_module):
        f = trainer._fused
        if not self.want:
            assert f is None
            return
        assert isinstance(f, GraphedTrainStep) and not f.failed, getattr(f, "reason", None)
        assert f.steps_done == trainer.global_step
        if self.horovod:
            assert getattr(f, "horovod_adopted", False) and trainer.accelerator_backend.sync is not None


@pytest.mark.parametrize("kind", ["ddp", "horovod"])
def test_graph_body_world2_matches_eager(tmpdir, kind):
    """World 2 (gloo, runtime actors): the graph-step body -- for Horovod with the
    DistributedOptimizer's reduction adopted by the DDP GradSynchronizer (the
    capturable form) -- trains exactly like the eager accelerator path."""
    from ray_lightning_accelerators_amd import HorovodRayAccelerator, RayAccelerator
    from ray_lightning_accelerators_amd import runtime as ray

    outs = {}
    ray.init(num_cpus=2, num_gpus=0)
    try:
        for graph in (True, False):
            m = _Dist()
            m.hip_graph_step = graph
            acc = (RayAccelerator(num_workers=2, use_gpu=False) if kind == "ddp"
                   else HorovodRayAccelerator(num_slots=2, use_gpu=False))
            t = pl.Trainer(default_root_dir=os.path.join(str(tmpdir), f"{kind}{graph}"), max_epochs=2,
                           progress_bar_refresh_rate=0, accelerator=acc,
                           callbacks=[_AssertGraphStep(graph, kind == "horovod")])
            assert t.fit(m) == 1
            outs[graph] = {k: v.clone() for k, v in m.state_dict().items()}
    finally:
        ray.shutdown()
    for k in outs[True]:
        assert torch.equal(outs[True][k], outs[False][k]), k
