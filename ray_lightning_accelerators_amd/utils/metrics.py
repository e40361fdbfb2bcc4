"""Observability: per-rank step-time / throughput counters
aggregated across workers, and a Prometheus exporter.

The reference has no metrics channel besides Tune reporting (``tune.py:97-101``)
and PL's rank-local loggers.  Here:

* :class:`ThroughputMonitor` times every training step on every rank (HIP
  events on GPU -- no host sync inside the epoch -- wall clock on CPU), and at
  each epoch end gathers the per-rank summaries (``all_gather_object`` over
  the job's process group) so rank 0 can publish whole-job samples/sec, the
  step-time p50/p99 and the slowest rank (straggler detection) into
  ``trainer.callback_metrics`` -- which the Tune callbacks and loggers read.
* :class:`PrometheusExporter` serves ``callback_metrics`` (and the monitor's
  numbers) as gauges on an HTTP ``/metrics`` endpoint from rank 0
  (``prometheus_client``; one registry per exporter).
"""
from __future__ import annotations

import re
import time
from typing import Dict, List, Optional

import torch

from ..lightning.callbacks import Callback
from .profiling import gather_summaries


def _batch_size(batch) -> int:
    if isinstance(batch, torch.Tensor):
        return int(batch.size(0)) if batch.dim() else 1
    if isinstance(batch, (list, tuple)) and batch:
        return _batch_size(batch[0])
    if isinstance(batch, dict) and batch:
        return _batch_size(next(iter(batch.values())))
    return 0


class ThroughputMonitor(Callback):
    """Per-rank step timing + cross-rank aggregation at every train epoch end.

    Publishes (rank 0, in ``trainer.callback_metrics``):
    ``perf/samples_per_sec`` (whole job), ``perf/step_ms_p50``, ``perf/step_ms_p99``,
    ``perf/step_ms_max_rank`` (mean step time of the slowest rank) and
    ``perf/straggler_rank``.  ``history`` keeps one dict per epoch on every rank.
    """

    def __init__(self, use_events: Optional[bool] = None):
        self.use_events = use_events
        self.history: List[Dict[str, float]] = []
        self._reset()

    def _reset(self) -> None:
        self._events: List[torch.cuda.Event] = []
        self._times: List[float] = []
        self._weights: List[int] = []  # steps covered by each marked interval
        self._samples = 0

    def _gpu(self, pl_module) -> bool:
        if self.use_events is not None:
            return bool(self.use_events) and torch.cuda.is_available()
        try:
            return next(pl_module.parameters()).is_cuda
        except StopIteration:
            return False

    def _mark(self, gpu: bool) -> None:
        if gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._events.append(ev)
        else:
            self._times.append(time.perf_counter())

    def on_train_epoch_start(self, trainer, pl_module):
        self._reset()
        self._mark(self._gpu(pl_module))

    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx, dataloader_idx):
        self._samples += _batch_size(batch)
        self._mark(self._gpu(pl_module))
        self._weights.append(1)

    def on_train_chunk_end(self, trainer, pl_module, outputs, n_steps, n_samples):
        """Multi-step dispatch (Trainer ``steps_per_dispatch``): one mark per chunk;
        per-step times are the chunk's mean."""
        self._samples += int(n_samples)
        self._mark(self._gpu(pl_module))
        self._weights.append(max(1, int(n_steps)))

    def _local(self) -> Dict[str, float]:
        if len(self._events) >= 2:
            torch.cuda.synchronize()
            d = [a.elapsed_time(b) for a, b in zip(self._events[:-1], self._events[1:])]
        else:
            d = [1e3 * (b - a) for a, b in zip(self._times[:-1], self._times[1:])]
        if not d:
            return {"steps": 0.0, "samples": float(self._samples), "total_ms": 0.0}
        t = torch.tensor(d, dtype=torch.float64)
        w = torch.tensor((self._weights + [1] * len(d))[: len(d)], dtype=torch.float64)
        per = t / w
        return {"steps": float(w.sum()), "samples": float(self._samples), "total_ms": float(t.sum()),
                "mean_ms": float(t.sum() / w.sum()), "p50_ms": float(per.median()),
                "p99_ms": float(torch.quantile(per, 0.99)), "max_ms": float(per.max())}

    def on_train_epoch_end(self, trainer, pl_module, outputs=None):
        ranks = gather_summaries(self._local())
        timed = [r for r in ranks if r.get("steps", 0) > 0]
        out: Dict[str, float] = {"epoch": float(trainer.current_epoch), "ranks": float(len(ranks))}
        if timed:
            # whole job: every rank's samples over the slowest rank's epoch time
            slowest = max(range(len(ranks)), key=lambda i: ranks[i].get("total_ms", 0.0))
            wall_ms = ranks[slowest]["total_ms"]
            out.update({
                "samples_per_sec": sum(r["samples"] for r in ranks) / max(wall_ms / 1e3, 1e-9),
                "step_ms_p50": sorted(r["p50_ms"] for r in timed)[len(timed) // 2],
                "step_ms_p99": max(r["p99_ms"] for r in timed),
                "step_ms_max_rank": ranks[slowest].get("mean_ms", 0.0),
                "straggler_rank": float(slowest),
            })
        self.history.append(out)
        if getattr(trainer, "global_rank", 0) == 0:
            for k, v in out.items():
                trainer.callback_metrics[f"perf/{k}"] = torch.tensor(v)


_NAME = re.compile(r"[^a-zA-Z0-9_]")


def metric_name(key: str, prefix: str = "rla_") -> str:
    return prefix + _NAME.sub("_", key).strip("_")


class PrometheusExporter(Callback):
    """Serve ``trainer.callback_metrics`` as Prometheus gauges from rank 0.

    ``port=0`` picks a free port (``self.port`` after ``on_fit_start``).  Gauges
    refresh every ``every_n_steps`` training steps and at every epoch end.
    """

    def __init__(self, port: int = 0, addr: str = "127.0.0.1", every_n_steps: int = 50):
        self.port, self.addr, self.every = int(port), addr, max(1, int(every_n_steps))
        self._server = None
        self._gauges = {}
        self.registry = None

    def __getstate__(self):  # the HTTP server never travels to the workers
        d = dict(self.__dict__)
        d["_server"], d["_gauges"], d["registry"] = None, {}, None
        return d

    def on_fit_start(self, trainer, pl_module):
        if getattr(trainer, "global_rank", 0) != 0 or self._server is not None:
            return
        from prometheus_client import CollectorRegistry, start_http_server

        self.registry = CollectorRegistry()
        self._server, _ = start_http_server(self.port, addr=self.addr, registry=self.registry)
        self.port = self._server.server_address[1]
        self._gauge("global_step", trainer.global_step)

    def _gauge(self, key: str, value) -> None:
        from prometheus_client import Gauge

        try:
            v = float(value.item() if isinstance(value, torch.Tensor) else value)
        except (TypeError, ValueError, RuntimeError):
            return
        name = metric_name(key)
        g = self._gauges.get(name)
        if g is None:
            g = self._gauges[name] = Gauge(name, f"ray_lightning_accelerators_amd metric {key}",
                                           registry=self.registry)
        g.set(v)

    def _publish(self, trainer) -> None:
        if self._server is None:
            return
        self._gauge("global_step", trainer.global_step)
        self._gauge("epoch", trainer.current_epoch)
        for k, v in list(trainer.callback_metrics.items()):
            if isinstance(v, torch.Tensor) and v.numel() != 1:
                continue
            self._gauge(k, v)

    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx, dataloader_idx):
        if self._server is not None and (trainer.global_step + 1) % self.every == 0:
            self._publish(trainer)

    def on_train_chunk_end(self, trainer, pl_module, outputs, n_steps, n_samples):
        # the Trainer already advanced global_step by the chunk
        if self._server is not None and \
                trainer.global_step // self.every != (trainer.global_step - int(n_steps)) // self.every:
            self._publish(trainer)

    def on_train_epoch_end(self, trainer, pl_module, outputs=None):
        self._publish(trainer)

    def on_validation_end(self, trainer, pl_module):
        self._publish(trainer)

    def close(self) -> None:
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None
