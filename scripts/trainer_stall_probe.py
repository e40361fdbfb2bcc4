"""Diagnostic: where does a slow Trainer epoch's time go?  Runs Trainer.fit of
MNISTClassifier in-process on one GPU and times (device-synced) each epoch's
sampler-order upload, every dispatch chunk (capture vs replay), and Python GC
pauses; prints one JSON row per epoch."""
import gc
import json
import sys
import tempfile
import time

import torch

sys.path.insert(0, ".")
import ray_lightning_accelerators_amd.lightning as pl  # noqa: E402
from ray_lightning_accelerators_amd.models import mnist  # noqa: E402

rows = {}
cur = {"epoch": -1}
gcs = []


def now():
    if not torch.cuda.is_current_stream_capturing():
        torch.cuda.synchronize()
    return time.perf_counter()


def wrap(cls, name, tag):
    orig = getattr(cls, name)

    def f(self, *a, **k):
        t0 = now()
        cap = getattr(self, "eng", None) is not None and self.eng._graph is None
        out = orig(self, *a, **k)
        dt = now() - t0
        r = rows.setdefault(cur["epoch"], {"chunks": [], "captures": 0})
        if tag == "chunk":
            r["chunks"].append(round(dt * 1e3, 3))
            if cap and self.eng._graph is not None:
                r["captures"] += 1
        else:
            r[tag] = round(dt * 1e3, 3)
        return out
    setattr(cls, name, f)


from ray_lightning_accelerators_amd.parallel import mlp_engine  # noqa: E402

def train_chunk_timed(self, n_steps, graph_steps=8):
    """FusedMNISTStep.train_chunk with a synced timestamp after every statement."""
    from ray_lightning_accelerators_amd.config import get_config

    marks = [("start", now())]
    eng = self.eng
    self._sync_lr()
    g = self.opt.param_groups[0]
    eng.lr, eng.betas, eng.eps, eng.wd = self.lr_val, tuple(g["betas"]), g["eps"], g["weight_decay"]
    marks.append(("prologue", now()))
    done = 0
    if graph_steps > 1 and eng._graph is None and not self._capture_failed and get_config().use_hip_graph \
            and n_steps > graph_steps and eng.steps_to_epoch_end() > graph_steps:
        self._capture_failed = not eng.capture(graph_steps)
        done = 1
    marks.append(("capture", now()))
    eng.run(n_steps - done)
    marks.append(("run", now()))
    first = self.gs.step
    self.gs.step += n_steps
    for q in g["params"]:
        st = self.opt.state.get(q)
        if st is not None and "step" in st:
            st["step"].fill_(float(self.gs.step))
    marks.append(("opt_state_fill", now()))
    ring = eng.stats.size(0)
    k = min(n_steps, ring)
    slots = (torch.arange(k, device=self.dev) + (first + n_steps - k)) % ring
    rows_ = eng.stats.index_select(0, slots)
    marks.append(("stats_gather", now()))
    last = rows_[-1]
    self.model.log("ptl/train_loss", last[0])
    self.model.log("ptl/train_accuracy", last[1] / last[2].clamp(min=1))
    self.trainer.callback_metrics["loss"] = last[0]
    marks.append(("log", now()))
    out = [{"loss": rows_[i, 0]} for i in range(k)]
    marks.append(("outputs", now()))
    r = rows.setdefault(cur["epoch"], {"chunks": [], "captures": 0})
    worst = r.setdefault("worst_stmt", ("", 0.0))
    for (a, ta), (b, tb) in zip(marks, marks[1:]):
        if (tb - ta) * 1e3 > worst[1]:
            r["worst_stmt"] = worst = (b, round((tb - ta) * 1e3, 3))
    return out


mnist.FusedMNISTStep.train_chunk = train_chunk_timed
wrap(mnist.FusedMNISTStep, "train_chunk", "chunk")


def wrap_max(cls, name, tag):
    orig = getattr(cls, name)

    def f(self, *a, **k):
        t0 = now()
        out = orig(self, *a, **k)
        dt = (now() - t0) * 1e3
        r = rows.setdefault(cur["epoch"], {"chunks": [], "captures": 0})
        r[tag + "_max_ms"] = round(max(r.get(tag + "_max_ms", 0.0), dt), 3)
        r[tag + "_n"] = r.get(tag + "_n", 0) + 1
        return out
    setattr(cls, name, f)


wrap_max(mlp_engine.FusedMLPEngine, "prime", "prime")
wrap_max(mlp_engine.FusedMLPEngine, "_device_step", "device_step")
wrap_max(mlp_engine.FusedMLPEngine, "begin_epoch", "begin_epoch")
wrap_max(mlp_engine.FusedMLPEngine, "_advance_host", "advance_host")
wrap_max(torch.cuda.CUDAGraph, "replay", "replay")
wrap(mnist.FusedMNISTStep, "make_epoch_batches", "epoch_batches_ms")
wrap(mnist.FusedMNISTStep, "eval_epoch", "eval_ms")


def gc_cb(phase, info):
    if phase == "start":
        gc_cb.t0 = time.perf_counter()
    else:
        gcs.append((cur["epoch"], info.get("generation"), round((time.perf_counter() - gc_cb.t0) * 1e3, 3)))


gc.callbacks.append(gc_cb)


class Ep(pl.Callback):
    def on_train_epoch_start(self, trainer, m):
        cur["epoch"] = trainer.current_epoch


model = mnist.MNISTClassifier({"layer_1": 32, "layer_2": 64, "lr": 0.1, "batch_size": 32})
tr = pl.Trainer(default_root_dir=tempfile.mkdtemp(), max_epochs=6, gpus=1, progress_bar_refresh_rate=0,
                callbacks=[Ep()])
tr.fit(model)
for e, r in sorted(rows.items()):
    ch = r["chunks"]
    r["n_chunks"] = len(ch)
    r["first_chunks_ms"] = ch[:3]
    r["max_chunk_ms"] = max(ch) if ch else None
    r["sum_chunks_ms"] = round(sum(ch), 3)
    del r["chunks"]
    r["gc"] = [g for g in gcs if g[0] == e]
    print(json.dumps({"epoch": e, **r}), flush=True)
