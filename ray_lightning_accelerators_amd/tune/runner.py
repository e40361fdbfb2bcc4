"""Trial runner: ``tune.run`` over the built-in actor runtime.

Each trial is an actor process that runs the trainable; the trainable's own
training workers (e.g. ``RayAccelerator(num_workers=2)``) are nested actors.
Resource accounting follows Ray Tune's ``resources_per_trial`` convention:
a trial is started only when ``cpu + extra_cpu`` CPUs and ``gpu + extra_gpu``
GPUs are free in the cluster ledger, so e.g. 4 trials x 2 GPU-workers pack
onto one 8 x MI355X node (BASELINE.json config 4).  Reports stream back to
the driver through a 0-CPU queue actor, which also lets schedulers (ASHA)
stop trials early.
"""
from __future__ import annotations

import json
import os
import sys
import time
import traceback
import uuid
from typing import Any, Callable, Dict, List, Optional, Union

from .. import runtime
from ..runtime.queue import Queue
from . import session as tsession
from .analysis import ExperimentAnalysis, Trial
from .sample import generate_variants
from .schedulers import FIFOScheduler, TrialScheduler
from ..utils.timeline import mark


TRIAL_REUSE_KEY = "rla-tune-trial"


class _TrialActor:
    """Runs one trial's trainable inside its own process.  With
    ``config.reuse_workers`` the process is recycled for the next trial (the
    runtime parks it instead of ending it), so trials after the first skip the
    interpreter + torch start-up."""

    def __rla_park__(self) -> None:
        # undo what run() changed in the process (the head's assignment resets the
        # environment, working directory and log descriptors)
        for name in ("stdout", "stderr"):
            cur, orig = getattr(sys, name), getattr(sys, f"__{name}__")
            if cur is not orig:
                try:
                    cur.close()
                except Exception:  # noqa: BLE001
                    pass
                setattr(sys, name, orig)
        tsession.shutdown_trial_session()

    def run(self, fn: Callable, config: Dict[str, Any], trial_id: str, trial_dir: str, report_queue,
            experiment_id: str, log_to_file: bool) -> Dict[str, Any]:
        os.makedirs(trial_dir, exist_ok=True)
        os.chdir(trial_dir)
        if log_to_file:
            sys.stdout = open(os.path.join(trial_dir, "stdout"), "a", buffering=1)
            sys.stderr = open(os.path.join(trial_dir, "stderr"), "a", buffering=1)
        from ..utils.timeline import mark

        mark("trial_start", trial=trial_id)
        tsession.init_trial_session(trial_id, trial_dir, config, report_queue, experiment_id)
        try:
            fn(config)
        finally:
            tsession.shutdown_trial_session()
            mark("trial_end", trial=trial_id)
        return {"ok": True}


def _normalize_resources(res: Optional[Dict[str, Any]]) -> Dict[str, float]:
    res = dict(res or {})
    cpu = float(res.get("cpu", 1))
    gpu = float(res.get("gpu", 0))
    return {"cpu": cpu, "gpu": gpu, "extra_cpu": float(res.get("extra_cpu", 0)),
            "extra_gpu": float(res.get("extra_gpu", 0)), "custom": res.get("custom_resources", {})}


def _should_stop(stop, trial_id: str, result: Dict[str, Any]) -> bool:
    if stop is None:
        return False
    if callable(stop):
        return bool(stop(trial_id, result))
    for k, v in stop.items():
        if k in result and result[k] >= v:
            return True
    return False


def run(
    run_or_experiment: Union[Callable, str],
    name: Optional[str] = None,
    metric: Optional[str] = None,
    mode: Optional[str] = None,
    stop: Optional[Union[Dict[str, Any], Callable]] = None,
    config: Optional[Dict[str, Any]] = None,
    resources_per_trial: Optional[Dict[str, Any]] = None,
    num_samples: int = 1,
    local_dir: Optional[str] = None,
    scheduler: Optional[TrialScheduler] = None,
    search_alg: Any = None,
    verbose: int = 1,
    log_to_file: bool = False,
    max_concurrent_trials: Optional[int] = None,
    raise_on_failed_trial: bool = True,
    fail_fast: bool = False,
    seed: Optional[int] = None,
    **kwargs,
) -> ExperimentAnalysis:
    if not callable(run_or_experiment):
        raise TypeError("only function trainables are supported")
    if not runtime.is_initialized():
        runtime.init()
    fn = run_or_experiment
    fname = getattr(fn, "__name__", "trainable")
    local_dir = os.path.expanduser(local_dir or os.environ.get("TUNE_RESULT_DIR", "~/ray_results"))
    exp_name = name or f"{fname}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
    exp_dir = os.path.join(local_dir, exp_name)
    os.makedirs(exp_dir, exist_ok=True)
    experiment_id = uuid.uuid4().hex
    res = _normalize_resources(resources_per_trial)
    need_cpu = res["cpu"] + res["extra_cpu"]
    need_gpu = res["gpu"] + res["extra_gpu"]
    total = runtime.cluster_resources()
    if need_cpu > total.get("CPU", 0) + 1e-9 or need_gpu > total.get("GPU", 0) + 1e-9:
        raise ValueError(f"trial needs {need_cpu} CPU / {need_gpu} GPU but the cluster has {total}")
    configs = generate_variants(config or {}, num_samples, seed=seed)
    trials = [Trial(trial_id=f"{uuid.uuid4().hex[:5]}_{i:05d}", config=c, index=i) for i, c in enumerate(configs)]
    for t in trials:
        t.logdir = os.path.join(exp_dir, f"{fname}_{t.trial_id}")
        os.makedirs(t.logdir, exist_ok=True)
        with open(os.path.join(t.logdir, "params.json"), "w") as f:
            json.dump(t.config, f, default=repr)
    scheduler = scheduler or FIFOScheduler()
    scheduler.set_search_properties(metric, mode)
    if need_gpu > 0:
        from ..config import GPU_WORKER_REUSE_KEY, get_config

        if get_config().reuse_workers:
            # one recycled GPU worker per free GPU, warming up (HIP context, native
            # kernels) while the first trial processes start: the trials' training
            # workers then skip that start-up, and every later trial reuses them
            try:
                runtime.prewarm_gpu_workers(GPU_WORKER_REUSE_KEY)
            except Exception:  # noqa: BLE001 - an optimisation only
                pass
    reports = Queue(actor_options={"num_cpus": 0})
    trial_cls = runtime.ActorClass(_TrialActor)
    from ..config import get_config

    trial_opts = {"_reuse": TRIAL_REUSE_KEY} if get_config().reuse_workers else {}
    pending = list(trials)
    running: Dict[str, Trial] = {}
    used_cpu = used_gpu = 0.0
    by_id = {t.trial_id: t for t in trials}
    failures = []

    def _on_result(trial_id: str, result: Dict[str, Any]) -> None:
        t = by_id.get(trial_id)
        if t is None or t.status != "RUNNING":
            return
        ckpt = result.pop("_checkpoint", None)
        result["config"] = t.config
        t.add_result(result, ckpt)
        decision = scheduler.on_trial_result(t, result)
        if _should_stop(stop, trial_id, result) or decision == TrialScheduler.STOP:
            t.stop_requested = True
    try:
        while pending or running:
            # launch what fits
            while pending and (max_concurrent_trials is None or len(running) < max_concurrent_trials):
                if used_cpu + need_cpu > total.get("CPU", 0) + 1e-9 or used_gpu + need_gpu > total.get("GPU", 0) + 1e-9:
                    break
                t = pending.pop(0)
                actor = trial_cls.options(num_cpus=res["cpu"], num_gpus=res["gpu"],
                                          resources=res["custom"] or None, **trial_opts).remote()
                t.actor = actor
                t.future = actor.run.remote(fn, t.config, t.trial_id, t.logdir, reports, experiment_id, log_to_file)
                t.status = "RUNNING"
                t.start_time = time.time()
                running[t.trial_id] = t
                used_cpu += need_cpu
                used_gpu += need_gpu
                scheduler.on_trial_add(t)
            # results
            # short wait: a finished trial is noticed (and its resources re-used by
            # the next) within ~20 ms instead of a fixed 0.2 s poll period
            for trial_id, result in reports.get_blocking_batch(timeout=0.02):
                _on_result(trial_id, result)
            # completions
            for tid, t in list(running.items()):
                done = t.future.done()
                if not done and not t.stop_requested:
                    continue
                if done:
                    # reports the trial queued before returning may still be in flight:
                    # take them (every trial's, in queue order) before it is released
                    for trial_id, result in reports.drain():
                        _on_result(trial_id, result)
                    try:
                        runtime.get(t.future)
                        t.status = "TERMINATED"
                    except Exception as e:  # noqa: BLE001
                        t.status = "ERROR"
                        t.error = "".join(traceback.format_exception_only(type(e), e))
                        failures.append(t)
                        if verbose:
                            print(f"Trial {tid} errored: {t.error[:2000]}", file=sys.stderr)
                else:
                    t.status = "TERMINATED"
                mark("trial_reaped", trial=tid)
                runtime.kill(t.actor)
                mark("trial_actor_released", trial=tid)
                t.end_time = time.time()
                del running[tid]
                used_cpu -= need_cpu
                used_gpu -= need_gpu
                scheduler.on_trial_complete(t, t.last_result)
                if fail_fast and t.status == "ERROR":
                    for p in pending:
                        p.status = "TERMINATED"
                    pending = []
    finally:
        for t in list(running.values()):
            try:
                runtime.kill(t.actor)
            except Exception:
                pass
        reports.shutdown()
    for t in trials:
        t.write_logs()
    if failures and raise_on_failed_trial:
        raise RuntimeError(f"{len(failures)} trial(s) failed: " + "; ".join(t.error or "?" for t in failures)[:4000])
    return ExperimentAnalysis(exp_dir, trials, default_metric=metric, default_mode=mode)


def with_parameters(trainable: Callable, **kwargs) -> Callable:
    """Bind large constant arguments to a trainable (they travel once, with it)."""
    def inner(config):
        return trainable(config, **kwargs)

    inner.__name__ = getattr(trainable, "__name__", "trainable")
    return inner
