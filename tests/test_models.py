"""Workload models: ResNet-50 (BASELINE config 5) definition and a tiny CPU
training run through the Trainer + flat arena + fused SGD path."""
import pytest
import torch

from ray_lightning_accelerators_amd import lightning as pl
from ray_lightning_accelerators_amd.models.resnet import (RESNET50_PARAMS, LightningResNet50, SyntheticImageNet,
                                                          resnet50)


def test_resnet50_shape_and_param_count():
    m = resnet50()
    assert sum(p.numel() for p in m.parameters()) == RESNET50_PARAMS
    assert len(list(m.parameters())) == 161
    out = m(torch.randn(2, 3, 64, 64))
    assert out.shape == (2, 1000)


def test_synthetic_imagenet_deterministic():
    ds = SyntheticImageNet(4, image_size=32, num_classes=10, seed=3)
    a, ya = ds[2]
    b, yb = ds[2]
    assert torch.equal(a, b) and ya == yb and a.shape == (3, 32, 32) and 0 <= ya < 10


def test_resnet50_trainer_cpu(tmpdir):
    model = LightningResNet50({"image_size": 32, "num_classes": 10, "batch_size": 4, "n_train": 8, "lr": 0.01})
    before = [p.detach().clone() for p in model.parameters()]
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=2,
                         checkpoint_callback=False)
    assert trainer.fit(model) == 1
    changed = sum(int(not torch.equal(a, b)) for a, b in zip(before, model.parameters()))
    assert changed > 100
    assert torch.isfinite(torch.as_tensor(float(trainer.callback_metrics["train_loss"])))


def test_resnet50_trainer_validation_cpu(tmpdir):
    """the config-5 module validates every epoch -- held-out loss
    and top-1 in callback_metrics, finite."""
    model = LightningResNet50({"image_size": 32, "num_classes": 10, "batch_size": 4, "n_train": 8, "n_val": 8,
                               "lr": 0.01})
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=2, checkpoint_callback=False,
                         num_sanity_val_steps=0)
    assert trainer.fit(model) == 1
    assert trainer.num_val_batches == [2]
    for k in ("val_loss", "val_acc"):
        v = float(trainer.callback_metrics[k])
        assert v == v and abs(v) != float("inf"), (k, v)
    assert 0.0 <= float(trainer.callback_metrics["val_acc"]) <= 1.0


@pytest.mark.gpu
def test_resnet50_resident_validation_matches_loader(tmpdir):
    """On the GPU the captured Trainer step gathers validation batches from the
    resident set (no per-image CPU work); the metrics equal iterating the loader."""
    from ray_lightning_accelerators_amd.lightning.graph_step import GraphedTrainStep

    cfg = {"image_size": 32, "num_classes": 10, "batch_size": 8, "n_train": 32, "n_val": 20, "lr": 0.01}
    model = LightningResNet50(cfg)
    trainer = pl.Trainer(default_root_dir=str(tmpdir), gpus=1, max_epochs=1, checkpoint_callback=False,
                         num_sanity_val_steps=0)
    assert trainer.fit(model) == 1
    assert isinstance(trainer._fused, GraphedTrainStep) and trainer._fused._eval_resident
    got = (float(trainer.callback_metrics["val_loss"]), float(trainer.callback_metrics["val_acc"]))
    # the same weights through the loader path (3 batches, the last one partial)
    model.eval()
    dl = model.val_dataloader()
    losses, accs = [], []
    with torch.no_grad():
        for i, (x, y) in enumerate(dl):
            out = model.validation_step((x.cuda(), y.cuda()), i)
            losses.append(out["val_loss"])
            accs.append(out["val_acc"])
    want = (float(torch.stack(losses).mean()), float(torch.stack(accs).mean()))
    assert abs(got[0] - want[0]) < 1e-3 * max(1.0, abs(want[0])) and abs(got[1] - want[1]) < 1e-6, (got, want)


@pytest.mark.gpu
def test_resnet50_gpu_step_bf16():
    """One fused-optimizer training step on the GPU (NHWC, bf16 autocast)."""
    import torch.nn.functional as F

    from ray_lightning_accelerators_amd.parallel.arena import ParamArena
    from ray_lightning_accelerators_amd.parallel.fused_optim import fuse_optimizer

    dev = torch.device("cuda", 0)
    model = resnet50(10).to(dev).to(memory_format=torch.channels_last)
    arena = ParamArena(model)
    opt = fuse_optimizer(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9), arena)
    x = torch.randn(8, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    w0 = model.fc.weight.detach().clone()
    for _ in range(2):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad()
    torch.cuda.synchronize()
    assert torch.isfinite(loss) and not torch.equal(w0, model.fc.weight)
