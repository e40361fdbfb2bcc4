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


@pytest.mark.gpu
def test_batched_state_dict_transfer_matches_per_tensor():
    """trainer._to_cpu: one transfer per dtype, same values / shapes / dtypes / structure."""
    from ray_lightning_accelerators_amd.lightning.trainer import _to_cpu

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    w = torch.randn(3, 5, generator=g).to(dev)
    sd = {"state": {0: {"step": torch.tensor(7.0), "exp_avg": w * 2, "exp_avg_sq": torch.randn(4, generator=g).to(dev)},
                    1: {"idx": torch.arange(5, device=dev), "half": torch.randn(6, generator=g).to(dev).bfloat16()}},
          "param_groups": [{"lr": 0.1, "params": [0, 1]}], "w": w, "w_again": w, "empty": torch.zeros(0, device=dev),
          "scalar": torch.tensor(2.5, device=dev), "t": (w[:, 1],)}
    out = _to_cpu(sd)

    def check(a, b):
        if isinstance(a, torch.Tensor):
            assert b.device.type == "cpu" and b.dtype == a.dtype and b.shape == a.shape
            assert torch.equal(a.cpu(), b)
        elif isinstance(a, dict):
            assert a.keys() == b.keys()
            for k in a:
                check(a[k], b[k])
        elif isinstance(a, (list, tuple)):
            assert type(a) is type(b) and len(a) == len(b)
            for x, y in zip(a, b):
                check(x, y)
        else:
            assert a == b

    check(sd, out)


@pytest.mark.gpu
def test_batched_state_dict_pickles_at_raw_size():
    """the host leaves must not be views of one shared buffer, or
    cloudpickle (the worker -> driver return path) writes that buffer once per leaf."""
    import cloudpickle

    from ray_lightning_accelerators_amd.lightning.trainer import _to_cpu

    dev = torch.device("cuda", 0)
    sd = {f"w{i}": torch.full((1024,), float(i), device=dev) for i in range(100)}  # 100 x 4 KiB
    out = _to_cpu(sd)
    raw = 100 * 1024 * 4
    size = len(cloudpickle.dumps(out))
    assert size < 1.5 * raw, (size, raw)
    assert all(torch.equal(out[k], sd[k].cpu()) for k in sd)


def test_process_checkpoint_writer_matches_atomic_save(tmp_path):
    """The writer PROCESS (shared-memory hand-off, pickling + I/O off the training
    process) writes files identical in content to atomic_save, in submission order,
    with removals ordered after the writes they follow."""
    import os

    from ray_lightning_accelerators_amd.lightning.utilities import ProcessCheckpointWriter, atomic_save

    w = ProcessCheckpointWriter()
    ck = {"epoch": 3, "state_dict": {"w": torch.randn(10, 5), "b": torch.arange(5), "e": torch.zeros(0)},
          "optimizer_states": [{"state": {0: {"step": torch.tensor(2.0), "m": torch.ones(3, dtype=torch.bfloat16)}},
                                "param_groups": [{"lr": 0.1, "params": [0]}]}], "hp": (1, "a")}
    for i in range(3):
        w.save(ck, str(tmp_path / f"c{i}.ckpt"))

    def _remove_file(p):
        os.remove(p)

    w.submit(_remove_file, str(tmp_path / "c0.ckpt"))
    w.wait()
    assert sorted(os.listdir(tmp_path)) == ["c1.ckpt", "c2.ckpt"]
    atomic_save(ck, str(tmp_path / "ref.ckpt"))
    a = torch.load(tmp_path / "c2.ckpt", weights_only=True)
    b = torch.load(tmp_path / "ref.ckpt", weights_only=True)
    assert a.keys() == b.keys() and a["hp"] == b["hp"] and a["epoch"] == 3
    for k in ck["state_dict"]:
        assert torch.equal(a["state_dict"][k], b["state_dict"][k])
    assert a["optimizer_states"][0]["state"][0]["m"].dtype == torch.bfloat16
    with pytest.raises(RuntimeError):
        w.save(ck, "/proc/definitely/not/writable.ckpt")
        w.wait()
    w.close()


def test_stalled_writer_process_is_taken_over(tmp_path, monkeypatch):
    """A writer process that stops answering (the Tune config-4 rehearsal once hung on
    it for good) is killed after STALL_S and its queued saves / removals complete in
    the training process, in order, only once the old process is gone; a fresh
    writer process takes the later saves (respawned, not dead for good)."""
    import os
    import signal

    from ray_lightning_accelerators_amd.lightning.utilities import ProcessCheckpointWriter, atomic_save

    monkeypatch.setattr(ProcessCheckpointWriter, "STALL_S", 1.0)
    w = ProcessCheckpointWriter()
    assert w._conn.poll(30)  # started
    old = w._proc
    os.kill(old.pid, signal.SIGSTOP)  # alive, silent

    def _remove_file(p):
        os.remove(p)

    try:
        ck = {"epoch": 1, "state_dict": {"w": torch.randn(4, 3)}}
        w.save(ck, str(tmp_path / "a.ckpt"))
        w.save(ck, str(tmp_path / "b.ckpt"))
        w.submit(_remove_file, str(tmp_path / "a.ckpt"))
        w.wait()  # returns after ~STALL_S instead of blocking forever
        assert sorted(os.listdir(tmp_path)) == ["b.ckpt"]
        assert not old.is_alive()  # stopped before anything was replayed
        assert w.alive() and w._proc.pid != old.pid  # a fresh writer process
        w.save(ck, str(tmp_path / "c.ckpt"))  # through the new writer
        w.wait()
        atomic_save(ck, str(tmp_path / "ref.ckpt"))
        assert torch.equal(torch.load(tmp_path / "c.ckpt", weights_only=True)["state_dict"]["w"],
                           torch.load(tmp_path / "ref.ckpt", weights_only=True)["state_dict"]["w"])
    finally:
        try:
            os.kill(old.pid, signal.SIGKILL)
        except OSError:
            pass
        w.close()


def test_busy_writer_heartbeats_are_not_a_stall(tmp_path, monkeypatch):
    """A save that takes longer than STALL_S (large checkpoint, slow filesystem) is
    busy, not stalled: the writer's heartbeats keep the trainer waiting for it."""
    from ray_lightning_accelerators_amd.lightning import utilities as u

    monkeypatch.setattr(u.ProcessCheckpointWriter, "STALL_S", 1.0)
    monkeypatch.setattr(u.ProcessCheckpointWriter, "BEAT_S", 0.2)
    w = u.ProcessCheckpointWriter()
    before = u.writer_takeovers
    try:
        assert w._conn.poll(30)
        w._conn.send(("sleep", 3.0))  # a test-only request: busy for 3 s
        w._pending.append((None, ("sleep", 3.0)))
        w.wait()
        assert u.writer_takeovers == before and w.alive()
    finally:
        w.close()


def test_process_writer_follows_cwd_changes(tmp_path, monkeypatch):
    """one writer process serves a recycled worker across fits / Tune
    trials that chdir into their own directory; relative checkpoint paths (and
    top-k removals) resolve against the TRAINING process's current directory."""
    import os

    from ray_lightning_accelerators_amd.lightning.utilities import ProcessCheckpointWriter

    w = ProcessCheckpointWriter()

    def _remove_file(p):
        os.remove(p)

    try:
        for trial in ("trial_a", "trial_b"):
            d = tmp_path / trial
            (d / "ckpt").mkdir(parents=True)
            monkeypatch.chdir(d)
            w.save({"epoch": 1, "w": torch.ones(3)}, os.path.join("ckpt", "e0.ckpt"))
            w.save({"epoch": 2, "w": torch.ones(3)}, os.path.join("ckpt", "e1.ckpt"))
            w.submit(_remove_file, os.path.join("ckpt", "e0.ckpt"))
            w.wait()
            assert sorted(os.listdir(d / "ckpt")) == ["e1.ckpt"], trial
    finally:
        w.close()


@pytest.mark.gpu
def test_deferred_checkpoints_match_inline(tmp_path, monkeypatch):
    """ModelCheckpoint's epoch-end save deferred to the background (device snapshot,
    decision once the monitored val_loss is known, no host sync at the epoch end)
    writes the same files with the same contents as the inline save of an
    identical, deterministic fit (fused MNIST step on the GPU)."""
    import torch

    from ray_lightning_accelerators_amd import lightning as pl
    from ray_lightning_accelerators_amd.lightning.callbacks import ModelCheckpoint
    from ray_lightning_accelerators_amd.lightning.utilities import load_checkpoint
    from ray_lightning_accelerators_amd.models.mnist import MNISTClassifier

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")

    def fit(defer: str, root):
        monkeypatch.setenv("RLA_DEFER_CKPT", defer)
        torch.manual_seed(0)
        model = MNISTClassifier({"layer_1": 32, "layer_2": 64, "lr": 1e-3, "batch_size": 32})
        ckpt = ModelCheckpoint(dirpath=str(root), save_last=True)
        trainer = pl.Trainer(default_root_dir=str(root), max_epochs=3, gpus=1, progress_bar_refresh_rate=0,
                             callbacks=[ckpt], limit_train_batches=120, limit_val_batches=20)
        assert trainer.fit(model) == 1
        deferred = getattr(trainer, "_deferred", None) is not None
        files = sorted(p.name for p in root.iterdir() if p.suffix == ".ckpt")
        return trainer, ckpt, files, deferred

    t_in, c_in, f_in, d_in = fit("0", tmp_path / "inline")
    t_df, c_df, f_df, d_df = fit("1", tmp_path / "deferred")
    assert not d_in and d_df, "the deferred path was not taken"
    assert f_in == f_df and "last.ckpt" in f_df
    assert os.path.basename(c_in.best_model_path) == os.path.basename(c_df.best_model_path)
    sa, sb = c_in.best_model_score, c_df.best_model_score
    assert (sa is None and sb is None) or float(sa) == float(sb)
    for name in f_in:
        a = load_checkpoint(str(tmp_path / "inline" / name))
        b = load_checkpoint(str(tmp_path / "deferred" / name))
        assert a["epoch"] == b["epoch"] and a["global_step"] == b["global_step"]
        # the callback state (PL 1.1: decided BEFORE the dump) agrees on both paths
        ca, cb = a["callbacks"]["ModelCheckpoint"], b["callbacks"]["ModelCheckpoint"]
        assert os.path.basename(ca["best_model_path"]) == os.path.basename(cb["best_model_path"]), name
        for k in ("best_model_score", "current_score"):
            assert (ca[k] is None and cb[k] is None) or float(ca[k]) == float(cb[k]), (name, k)
        if name != "last.ckpt":
            assert os.path.basename(cb["best_model_path"]) == name
        for k in a["state_dict"]:
            assert torch.equal(a["state_dict"][k], b["state_dict"][k]), (name, k)
        sa, sb = a["optimizer_states"][0]["state"], b["optimizer_states"][0]["state"]
        for i in sa:
            for k in sa[i]:
                assert torch.equal(torch.as_tensor(sa[i][k]), torch.as_tensor(sb[i][k])), (name, i, k)
    # the last checkpoint holds the final weights
    last = load_checkpoint(str(tmp_path / "deferred" / "last.ckpt"))
    for k, v in t_df.get_model().state_dict().items():
        assert torch.equal(last["state_dict"][k], v.detach().cpu()), k


def test_staged_state_is_a_snapshot():
    """_Staged (the deferred checkpoint's state) copies at staging time: later
    in-place updates -- Adam's CPU step counter, parameters -- do not leak into the
    host dict it produces, and its layout equals _to_cpu's."""
    from ray_lightning_accelerators_amd.lightning.trainer import _resolve_staged, _Staged, _to_cpu

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    w = torch.arange(6.0, device=dev).view(2, 3)
    b = torch.ones(3, device=dev, dtype=torch.float64)
    step = torch.tensor(5.0)
    sd = {"state": {0: {"exp_avg": w, "step": step}, 1: {"exp_avg": b}}, "param_groups": [{"lr": 0.1}],
          "w": w}
    expect = {k: v.clone() for k, v in _to_cpu({"w": w, "b": b}).items()}  # (CPU: _to_cpu aliases)
    staged = {"optimizer_states": [_Staged(sd)], "epoch": 3}
    w.add_(100.0)
    b.mul_(7.0)
    step.fill_(9.0)
    got = _resolve_staged(staged)
    assert got["epoch"] == 3
    host = got["optimizer_states"][0]
    assert torch.equal(host["state"][0]["exp_avg"], expect["w"])
    assert torch.equal(host["state"][1]["exp_avg"], expect["b"])
    assert float(host["state"][0]["step"]) == 5.0
    assert host["param_groups"] == [{"lr": 0.1}]
    assert host["state"][0]["exp_avg"].device.type == "cpu"
