"""Background checkpoint writer (lightning/utilities.py CheckpointWriter): writes
land in submission order, a removal queued after a write sees the file, the
written state is the snapshot taken at submit time, and errors surface at wait()."""
import os

import pytest
import torch

from ray_lightning_accelerators_amd.lightning.utilities import CheckpointWriter, load_checkpoint


def test_writes_snapshot_and_order(tmp_path):
    w = CheckpointWriter()
    t = torch.zeros(1000)
    p1, p2 = str(tmp_path / "a.ckpt"), str(tmp_path / "b.ckpt")
    w.save({"state_dict": {"w": t}, "epoch": 0}, p1)
    t.add_(1.0)  # the training loop keeps mutating its tensors after the submit
    w.save({"state_dict": {"w": t}, "epoch": 1}, p2)
    w.submit(os.remove, p1)  # top-k rotation: runs after the write of p1
    w.wait()
    assert not os.path.exists(p1)
    ck = load_checkpoint(p2)
    assert ck["epoch"] == 1 and torch.equal(ck["state_dict"]["w"], torch.ones(1000))
    w.close()


def test_snapshot_is_private(tmp_path):
    w = CheckpointWriter()
    t = torch.zeros(4)
    p = str(tmp_path / "c.ckpt")
    w.submit(lambda: None)
    w.save({"w": t}, p)
    t.fill_(7.0)
    w.wait()
    assert torch.equal(load_checkpoint(p)["w"], torch.zeros(4))
    w.close()


def test_error_surfaces_at_wait(tmp_path):
    w = CheckpointWriter()

    def boom():
        raise OSError("disk full")

    w.submit(boom)
    with pytest.raises(RuntimeError, match="disk full"):
        w.wait()
    w.close()
