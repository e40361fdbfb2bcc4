"""Tracing / profiling (the reference has none, PL 1.1 offers
``Trainer(profiler=...)`` per process).

* ``SimpleProfiler`` -- PL-compatible action timer (``profile(action)``
  context, ``summary()``).  With ``cuda_sync=True`` every action is bracketed
  by HIP events on the current stream, so the report is GPU time, not the
  host's asynchronous launch time.
* ``TorchProfiler`` -- wraps ``torch.profiler`` (roctracer on ROCm) for a
  window of steps and writes a chrome trace plus a kernel table: the
  hand-written kernels show up by name (``mlp3_head_kernel``,
  ``oneshot_allreduce_kernel``, ``adam_kernel`` ...).  For hardware counters
  use rocprofv3 (``scripts/profile_*.sh``).
* ``StepTimer`` -- per-step HIP-event timing of an engine loop, reduced to
  mean / p50 / p99 and aggregated across ranks with ``gather_summaries``.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch


class BaseProfiler:
    def start(self, action: str) -> None: ...

    def stop(self, action: str) -> None: ...

    @contextlib.contextmanager
    def profile(self, action: str):
        self.start(action)
        try:
            yield
        finally:
            self.stop(action)

    def summary(self) -> str:
        return ""

    def describe(self) -> None:
        s = self.summary()
        if s:
            print(s, flush=True)


class PassThroughProfiler(BaseProfiler):
    pass


class SimpleProfiler(BaseProfiler):
    def __init__(self, cuda_sync: bool = False):
        self.cuda_sync = cuda_sync and torch.cuda.is_available()
        self.recorded: Dict[str, List[float]] = defaultdict(list)
        self._open: Dict[str, object] = {}
        self._pending: List[tuple] = []  # (action, start_event, end_event)

    def start(self, action: str) -> None:
        if action in self._open:
            raise ValueError(f"profiler action {action!r} already started")
        if self.cuda_sync:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._open[action] = ev
        else:
            self._open[action] = time.perf_counter()

    def stop(self, action: str) -> None:
        t0 = self._open.pop(action, None)
        if t0 is None:
            raise ValueError(f"profiler action {action!r} was not started")
        if self.cuda_sync:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pending.append((action, t0, ev))
        else:
            self.recorded[action].append(time.perf_counter() - t0)

    def _flush(self) -> None:
        if self._pending:
            torch.cuda.synchronize()
            for action, a, b in self._pending:
                self.recorded[action].append(a.elapsed_time(b) / 1e3)
            self._pending = []

    def stats(self) -> Dict[str, Dict[str, float]]:
        self._flush()
        out = {}
        for k, v in self.recorded.items():
            t = torch.tensor(v, dtype=torch.float64)
            out[k] = {"calls": len(v), "total_s": float(t.sum()), "mean_ms": float(t.mean() * 1e3),
                      "p50_ms": float(t.median() * 1e3),
                      "p99_ms": float(torch.quantile(t, 0.99) * 1e3) if len(v) > 1 else float(t[0] * 1e3)}
        return out

    def summary(self) -> str:
        st = self.stats()
        if not st:
            return ""
        kind = "GPU (HIP events)" if self.cuda_sync else "host"
        lines = [f"Profiler report ({kind} time)", f"{'action':<32}{'calls':>8}{'mean ms':>12}{'p99 ms':>12}{'total s':>12}"]
        for k, s in sorted(st.items(), key=lambda kv: -kv[1]["total_s"]):
            lines.append(f"{k:<32}{s['calls']:>8}{s['mean_ms']:>12.4f}{s['p99_ms']:>12.4f}{s['total_s']:>12.4f}")
        return "\n".join(lines)


class TorchProfiler(BaseProfiler):
    """torch.profiler over the first ``active`` training batches after ``wait``."""

    def __init__(self, dirpath: Optional[str] = None, wait: int = 2, active: int = 10, row_limit: int = 25):
        self.dirpath = dirpath or os.path.join(os.getcwd(), "profiles")
        self.wait, self.active, self.row_limit = wait, active, row_limit
        self._prof = None
        self._n = 0
        self._table = ""

    def start(self, action: str) -> None:
        if action != "run_training_batch":
            return
        if self._prof is None and self._n == self.wait:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()

    def stop(self, action: str) -> None:
        if action != "run_training_batch":
            return
        self._n += 1
        if self._prof is not None and self._n >= self.wait + self.active:
            self._finish()

    def _finish(self) -> None:
        if self._prof is None:
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._prof.__exit__(None, None, None)
        os.makedirs(self.dirpath, exist_ok=True)
        rank = os.environ.get("RANK", os.environ.get("HOROVOD_RANK", "0"))
        self._prof.export_chrome_trace(os.path.join(self.dirpath, f"trace_rank{rank}.json"))
        key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        try:
            self._table = self._prof.key_averages().table(sort_by=key, row_limit=self.row_limit)
        except Exception:  # noqa: BLE001 - older builds name the column differently
            self._table = self._prof.key_averages().table(row_limit=self.row_limit)
        with open(os.path.join(self.dirpath, f"kernels_rank{rank}.txt"), "w") as f:
            f.write(self._table)
        self._prof = None

    def summary(self) -> str:
        self._finish()
        return self._table


def resolve_profiler(profiler) -> BaseProfiler:
    """Trainer(profiler=None | True | "simple" | "gpu" | "torch" | BaseProfiler)."""
    if profiler is None or profiler is False:
        return PassThroughProfiler()
    if isinstance(profiler, BaseProfiler):
        return profiler
    if profiler is True or profiler == "simple":
        return SimpleProfiler()
    if profiler == "gpu":
        return SimpleProfiler(cuda_sync=True)
    if profiler in ("torch", "advanced", "pytorch"):
        return TorchProfiler()
    raise ValueError(f"unknown profiler {profiler!r}")


class StepTimer:
    """HIP-event timing of consecutive steps without host syncs inside the loop."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._events: List[torch.cuda.Event] = []

    def mark(self) -> None:
        if self.enabled:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._events.append(ev)

    def summary(self) -> Dict[str, float]:
        if len(self._events) < 2:
            return {}
        torch.cuda.synchronize()
        d = torch.tensor([a.elapsed_time(b) for a, b in zip(self._events[:-1], self._events[1:])],
                         dtype=torch.float64)
        return {"steps": float(d.numel()), "mean_ms": float(d.mean()), "p50_ms": float(d.median()),
                "p99_ms": float(torch.quantile(d, 0.99)), "max_ms": float(d.max())}


def gather_summaries(summary: Dict[str, float]) -> List[Dict[str, float]]:
    """All ranks' summaries (rank order) via torch.distributed, or [summary]."""
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [summary]
    out: List[Optional[Dict[str, float]]] = [None] * dist.get_world_size()
    dist.all_gather_object(out, summary)
    return out  # type: ignore[return-value]
