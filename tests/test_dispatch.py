"""Multi-step dispatch of the fused resident step (Trainer ``steps_per_dispatch``).

CPU: a fake fused step records how the Trainer cuts each epoch into dispatches;
every chunk must end exactly where the per-batch loop does host work (logger
flush, validation point, max_steps, epoch end) and the run must see the same
global steps / validations as per-batch dispatch.  GPU: the real MNIST engine
trains bit-identically with hipGraph chunks and with one dispatch per batch.
"""
import pytest
import torch
from torch.utils.data import DataLoader

import ray_lightning_accelerators_amd.lightning as pl
from ray_lightning_accelerators_amd.lightning import Callback, LightningModule
from ray_lightning_accelerators_amd.models.data import RandomDataset
from ray_lightning_accelerators_amd.utils.metrics import ThroughputMonitor


class _FakeFused:
    max_chunk = 64

    def __init__(self, trainer):
        self.trainer = trainer
        self.chunks = []  # (global_step at start, steps)
        self.per_batch = 0
        self._B = 4

    def make_epoch_batches(self, dl, n):
        return [("__rla_resident__", i) for i in range(n)]

    def train_batch(self, batch, batch_idx):
        self.per_batch += 1
        return {"loss": torch.tensor(1.0)}

    def train_chunk(self, k):
        self.chunks.append((self.trainer.global_step, k))
        return [{"loss": torch.tensor(1.0)} for _ in range(k)]

    def sync_params_to_module(self):
        pass

    def load_params_from_module(self):
        pass


class _Model(LightningModule):
    def __init__(self):
        super().__init__()
        self.layer = torch.nn.Linear(32, 2)

    def forward(self, x):
        return self.layer(x)

    def training_step(self, batch, batch_idx):
        return self(batch).sum()

    def validation_step(self, batch, batch_idx):
        return {"x": self(batch).sum()}

    def configure_optimizers(self):
        return torch.optim.SGD(self.layer.parameters(), lr=0.1)

    def train_dataloader(self):
        return DataLoader(RandomDataset(32, 640), batch_size=4)

    def val_dataloader(self):
        return DataLoader(RandomDataset(32, 8), batch_size=4)

    def configure_fused_step(self, trainer):
        self.fake = _FakeFused(trainer)
        return self.fake


class _Count(Callback):
    def __init__(self):
        self.val_steps = []

    def on_validation_end(self, trainer, pl_module):
        self.val_steps.append(trainer.global_step)


class _BatchHook(Callback):
    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx, dataloader_idx):
        pass


def _fit(tmpdir, spd, callbacks=(), **kw):
    model = _Model()
    cnt = _Count()
    args = dict(max_epochs=2, val_check_interval=0.25, log_every_n_steps=50, num_sanity_val_steps=0,
                checkpoint_callback=False, progress_bar_refresh_rate=0)
    args.update(kw)
    tr = pl.Trainer(default_root_dir=str(tmpdir), steps_per_dispatch=spd, callbacks=[cnt, *callbacks], **args)
    assert tr.fit(model) == 1
    return tr, model.fake, cnt


def test_chunks_end_at_host_work_boundaries(tmpdir):
    tr, fake, cnt = _fit(tmpdir, 64)
    assert fake.per_batch == 0 and tr.global_step == 320
    n, every_val, every_log = 160, 40, 50
    gs = 0
    for start, k in fake.chunks:
        assert start == gs and 1 <= k <= 64
        b = start % n
        for i in range(1, k):  # no boundary strictly inside a chunk
            assert (b + i) % every_val != 0 and (gs + i) % every_log != 0, (start, k)
        end = b + k
        assert end == n or end % every_val == 0 or (gs + k) % every_log == 0 or k == 64, (start, k)
        gs += k
    assert gs == 320
    # same validations as one dispatch per batch
    tr1, fake1, cnt1 = _fit(tmpdir, 1)
    assert fake1.chunks == [] and fake1.per_batch == 320
    assert cnt.val_steps == cnt1.val_steps == [40, 80, 120, 160, 200, 240, 280, 320]


def test_max_steps_and_cap(tmpdir):
    tr, fake, _ = _fit(tmpdir, 16, max_steps=37, val_check_interval=1.0, log_every_n_steps=1000)
    assert tr.global_step == 37
    assert [k for _, k in fake.chunks] == [16, 16, 5]


def test_batch_hooks_disable_chunking_but_chunk_aware_callbacks_do_not(tmpdir):
    _, fake, _ = _fit(tmpdir, 64, callbacks=[_BatchHook()])
    assert fake.chunks == [] and fake.per_batch == 320
    mon = ThroughputMonitor(use_events=False)
    tr, fake, _ = _fit(tmpdir, 64, callbacks=[mon])
    assert fake.per_batch == 0 and fake.chunks
    assert mon.history[-1]["samples_per_sec"] > 0 and mon.history[-1]["step_ms_p50"] > 0


def test_step_scheduler_disables_chunking(tmpdir):
    class M(_Model):
        def configure_optimizers(self):
            opt = torch.optim.SGD(self.layer.parameters(), lr=0.1)
            return [opt], [{"scheduler": torch.optim.lr_scheduler.StepLR(opt, 10), "interval": "step"}]

    model = M()
    tr = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=20, num_sanity_val_steps=0,
                    checkpoint_callback=False, progress_bar_refresh_rate=0, steps_per_dispatch=64)
    assert tr.fit(model) == 1
    assert model.fake.chunks == [] and model.fake.per_batch == 20


@pytest.mark.gpu
def test_fused_mnist_chunked_dispatch_matches_per_batch(tmpdir):
    """hipGraph chunks of the real engine == one dispatch per batch, bit for bit."""
    from ray_lightning_accelerators_amd import ops
    from ray_lightning_accelerators_amd.models.mnist import LightningMNISTClassifier

    ops.require()
    res = {}
    for spd in (1, 64):
        pl.seed_everything(0)
        model = LightningMNISTClassifier({"layer_1": 32, "layer_2": 64, "lr": 1e-3, "batch_size": 32})
        tr = pl.Trainer(default_root_dir=str(tmpdir / f"s{spd}"), gpus=1, max_epochs=2, limit_train_batches=130,
                        limit_val_batches=2, checkpoint_callback=False, progress_bar_refresh_rate=0,
                        steps_per_dispatch=spd)
        assert tr.fit(model) == 1
        assert tr._fused is not None and tr._fused.eng is not None
        assert tr.global_step == 260
        if spd > 1:
            # the chunks (64, 64, 2 steps: they run across the log points, which the fused
            # step reports itself) are replays of the 64-step graph and the 1/2/.../32-step
            # remainder graphs
            assert tr._fused.eng._graph is not None and not tr._fused._capture_failed
            assert tr._fused.eng._graph_steps == 64 and sorted(tr._fused.eng._tail_graphs) == [1, 2, 4, 8, 16, 32]
        res[spd] = ({k: v.detach().cpu().clone() for k, v in model.state_dict().items()},
                    float(tr.callback_metrics["ptl/train_loss"]))
    for k, v in res[1][0].items():
        assert torch.equal(v, res[64][0][k]), k
    assert res[1][1] == res[64][1]


class _SpanFused(_FakeFused):
    """A fused step that reports its chunks' log points itself (like FusedMNISTStep)."""

    max_chunk = 2048
    chunk_spans_log_points = True

    def train_chunk(self, k):
        self.chunks.append((self.trainer.global_step, k))
        self._last_rows = torch.arange(k, dtype=torch.float32).unsqueeze(1).repeat(1, 4) + \
            float(self.trainer.global_step)
        self._last_rows[:, 2] = 1.0
        return [{"loss": torch.tensor(1.0)} for _ in range(k)]

    def log_points(self, rows, first, every):
        return [(first + 1 + i, {"ptl/train_loss": rows[i, 0], "ptl/train_accuracy": rows[i, 1] / rows[i, 2]})
                for i in range(rows.size(0)) if (first + 1 + i) % every == 0]


def test_chunks_span_log_points_when_the_fused_step_reports_them(tmpdir):
    """Chunks run across log points; every log point still reaches the logger under
    its own global step, with that step's values."""
    class M(_Model):
        def configure_fused_step(self, trainer):
            self.fake = _SpanFused(trainer)
            return self.fake

    model = M()
    tr = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, val_check_interval=1.0, log_every_n_steps=7,
                    num_sanity_val_steps=0, checkpoint_callback=False, progress_bar_refresh_rate=0,
                    steps_per_dispatch=1024)
    rows = []
    orig = tr.logger.log_metrics
    tr.logger.log_metrics = lambda metrics, step=None: (rows.append((step, dict(metrics))), orig(metrics, step))
    assert tr.fit(model) == 1
    assert model.fake.chunks == [(0, 160)]  # one dispatch for the epoch
    logged = [(st, m["ptl/train_loss"]) for st, m in rows if "ptl/train_loss" in m]
    # every log point (the validation-end flush writes the chunk's own last-step logs,
    # which this fake step does not make)
    assert [st for st, _ in logged] == list(range(7, 161, 7))
    for st, v in logged:
        assert float(v) == float(st - 1)  # row i of the chunk starting at step 0 holds i


@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [True, False])
@pytest.mark.parametrize("world,rank", [(1, 0), (3, 2), (8, 5)])
def test_sampler_order_matches_iteration(shuffle, drop_last, world, rank):
    """The fused path's tensor rebuild of a sampler's epoch order == iterating it."""
    from torch.utils.data import DistributedSampler, SequentialSampler

    from ray_lightning_accelerators_amd.models.mnist import _sampler_order

    ds = RandomDataset(4, 1003)
    s = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, drop_last=drop_last, seed=7)
    for epoch in (0, 3):
        s.set_epoch(epoch)
        assert torch.equal(_sampler_order(s), torch.tensor(list(iter(s)))), epoch
    q = SequentialSampler(ds)
    assert torch.equal(_sampler_order(q), torch.tensor(list(iter(q))))


@pytest.mark.parametrize("num_samples", [None, 500, 2500])
@pytest.mark.parametrize("with_generator", [False, True])
def test_random_sampler_order_matches_iteration(num_samples, with_generator):
    """RandomSampler (world size 1's shuffled loader): the tensor rebuild draws the
    same seed / permutations as iterating, and leaves the global RNG in the same state."""
    from torch.utils.data import RandomSampler

    from ray_lightning_accelerators_amd.models.mnist import _sampler_order

    ds = RandomDataset(4, 1003)

    def make():
        g = torch.Generator().manual_seed(11) if with_generator else None
        return RandomSampler(ds, num_samples=num_samples, generator=g)

    torch.manual_seed(5)
    a, b = make(), make()
    ref = [torch.tensor(list(iter(a))) for _ in range(2)]
    after_ref = torch.rand(3)
    torch.manual_seed(5)
    got = [_sampler_order(b) for _ in range(2)]
    after_got = torch.rand(3)
    for r, o in zip(ref, got):
        assert torch.equal(r, o)
    assert torch.equal(after_ref, after_got)
