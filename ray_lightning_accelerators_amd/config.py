"""Typed run-time configuration of the MI355X data plane.

The reference is configured by constructor kwargs only
(``ray_lightning/ray_ddp.py:79-83``, ``ray_horovod.py:82-87``) plus
``PL_GLOBAL_SEED`` (``ray_ddp.py:154-159``).  Those kwargs are kept unchanged;
the knobs that exist only because this framework owns its data plane live in
ONE dataclass, settable three ways (later wins):

1. defaults below,
2. environment ``RLA_<FIELD>`` (e.g. ``RLA_BUCKET_CAP_MB=4``),
3. explicit kwargs (``RayAccelerator(..., allreduce_algo="rccl")`` or
   ``RLAConfig.resolve(bucket_cap_mb=4)``).

The driver resolves the config once; it travels to the workers with the
accelerator and is installed there with :func:`set_config`, so every rank uses
the same values even when the workers' environments differ.  Rank 0 logs it
once at worker start (``describe``).
"""
from __future__ import annotations

import dataclasses
import logging
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, Optional

log = logging.getLogger(__name__)

ENV_PREFIX = "RLA_"

_CHOICES = {
    "grad_dtype": ("fp32", "bf16"),
    "allreduce_algo": ("auto", "oneshot", "twoshot", "rccl", "torch"),
    "precision": ("32", "bf16"),
    "pg_backend": ("auto", "nccl", "gloo"),
    "hip_graph_step": ("auto", "on", "off"),
}

# legacy env names kept working (first release used these spellings)
_ALIASES = {"fused_optimizer": "RLA_FUSED_OPTIM"}


@dataclass
class RLAConfig:
    """Data-plane knobs.  Every field maps to env ``RLA_<FIELD upper-case>``."""

    # DDP gradient bucket cap in MiB: large enough to amortise the ~us xGMI flag
    # barrier, small enough that the first bucket leaves early in backward
    bucket_cap_mb: float = 8.0
    # gradient wire dtype: bf16 halves the bytes on the 7 xGMI links
    grad_dtype: str = "fp32"
    # allreduce selection for fp32 buckets: auto = xGMI one-shot up to
    # ``xgmi_bytes``, xGMI two-shot up to ``twoshot_bytes``, RCCL above
    allreduce_algo: str = "auto"
    # one-shot receive area per rank (bytes); the MNIST gradient is 109-532 KiB
    xgmi_bytes: int = 2 << 20
    # largest bucket (bytes) of the xGMI two-shot (reduce-scatter + all-gather);
    # its region costs ~4x this per GPU (256 MiB of 288 GB); 0 disables two-shot
    twoshot_bytes: int = 64 << 20
    # native C++ communicator / reducer / Horovod fusion engine (else torch.distributed)
    native_comm: bool = True
    native_reducer: bool = True
    hvd_native: bool = True
    # fused single-launch HIP optimizers over the parameter arena
    fused_optimizer: bool = True
    # MNIST fused step: exchange gradients inside the tail kernel (world > 1)
    fused_dp: bool = True
    # capture the resident MNIST step into hipGraphs
    use_hip_graph: bool = True
    # Trainer: capture an autograd LightningModule's whole training step (forward,
    # backward, gradient all-reduce, fused optimizer) in one hipGraph and replay it
    # (lightning/graph_step.py).  auto = when the module sets hip_graph_step = True;
    # on = every module (host-reading steps still fall back); off = never
    hip_graph_step: str = "auto"
    # eager warm-up steps before the capture (allocator pools, MIOpen find, autotune)
    hip_graph_warmup: int = 3
    # ModelCheckpoint writes run in a writer PROCESS (state snapshot taken
    # synchronously into shared memory; pickling, file write and rename off this
    # process; the Trainer drains the writes before fit() returns).  Round 2's
    # writer thread was slower (GIL: MNIST epoch-end +0.7 ms, profiles/r2_c38).
    async_checkpoint: bool = True
    # RayAccelerator GPU workers are recycled across fits (Tune trials): a finished
    # fit parks its worker processes with their HIP context and loaded kernels, and
    # the next fit on the same GPUs takes them over (runtime actor reuse)
    reuse_workers: bool = True
    # the same recycling for CPU-only workers (off by default: a CPU worker starts
    # from the pre-warmed pool cheaply); used by the gloo tests of the reuse path
    reuse_cpu_workers: bool = False
    # Trainer: fused resident steps issued per host dispatch when nothing observes
    # single batches (chunks also end at validation / max_steps boundaries, and at log
    # points unless the fused step reports them itself); 1 = one dispatch per batch.
    # Capped by the fused step's stats ring (half of its 4,096 rows).
    steps_per_dispatch: int = 1024
    # torch.distributed backend of GPU workers: auto = RCCL ("nccl"); "gloo" only
    # for rehearsing N ranks on ONE device (RCCL refuses duplicate GPUs)
    pg_backend: str = "auto"
    # generic-model compute precision ("32" or "bf16" autocast)
    precision: str = "32"
    # bounded polls of the xGMI kernels (iterations) and the watchdog period (ms)
    # (2^27 polls with s_sleep: minutes -- long enough for a legitimately slow peer,
    # e.g. a rank still writing a checkpoint; a truly dead peer still ends the kernel)
    spin_limit: int = 1 << 27
    watchdog_ms: int = 100
    # debug: verify that every DDP bucket the comm stream reads equals what the
    # compute stream produced (stream-ordering race detector)
    check_streams: bool = False
    extra: Dict[str, Any] = field(default_factory=dict)

    # --------------------------------------------------------------- build
    def __post_init__(self) -> None:
        for k, allowed in _CHOICES.items():
            v = str(getattr(self, k))
            if v not in allowed:
                raise ValueError(f"{k}={v!r}: expected one of {allowed}")
            setattr(self, k, v)
        if self.bucket_cap_mb <= 0:
            raise ValueError("bucket_cap_mb must be > 0")

    @staticmethod
    def env_name(name: str) -> str:
        return ENV_PREFIX + name.upper()

    @classmethod
    def from_env(cls, environ: Optional[Dict[str, str]] = None) -> "RLAConfig":
        env = os.environ if environ is None else environ
        kw: Dict[str, Any] = {}
        for f in fields(cls):
            if f.name == "extra":
                continue
            for key in (cls.env_name(f.name), _ALIASES.get(f.name)):
                if key and key in env:
                    kw[f.name] = _parse(f.type, env[key], key)
                    break
        return cls(**kw)

    @classmethod
    def resolve(cls, **overrides) -> "RLAConfig":
        """defaults < env < explicit (non-None) kwargs."""
        cfg = cls.from_env()
        return cfg.replace(**{k: v for k, v in overrides.items() if v is not None})

    def replace(self, **kw) -> "RLAConfig":
        names = {f.name for f in fields(self)}
        bad = set(kw) - names
        if bad:
            raise TypeError(f"unknown config field(s): {sorted(bad)}")
        return dataclasses.replace(self, **kw)

    def to_env(self) -> Dict[str, str]:
        out = {}
        for f in fields(self):
            if f.name == "extra":
                continue
            v = getattr(self, f.name)
            out[self.env_name(f.name)] = ("1" if v else "0") if isinstance(v, bool) else str(v)
        return out

    def describe(self) -> str:
        items = ", ".join(f"{f.name}={getattr(self, f.name)!r}" for f in fields(self) if f.name != "extra")
        return f"RLAConfig({items})"


def _parse(typ, raw: str, key: str):
    t = typ if isinstance(typ, str) else getattr(typ, "__name__", str(typ))
    try:
        if t == "bool":
            low = raw.strip().lower()
            if low in ("1", "true", "yes", "on"):
                return True
            if low in ("0", "false", "no", "off", ""):
                return False
            raise ValueError(raw)
        if t == "int":
            return int(float(raw)) if "e" in raw.lower() else int(raw, 0)
        if t == "float":
            return float(raw)
        return raw
    except ValueError as e:
        raise ValueError(f"env {key}={raw!r} is not a valid {t}") from e


# runtime reuse key of RayAccelerator's GPU workers (recycled / pre-warmed processes)
GPU_WORKER_REUSE_KEY = "rla-ddp-gpu-worker"

_current: Optional[RLAConfig] = None


def get_config() -> RLAConfig:
    """The process's config: the one installed by the accelerator, else env."""
    global _current
    if _current is None:
        _current = RLAConfig.from_env()
    return _current


def set_config(cfg: Optional[RLAConfig]) -> None:
    """Install ``cfg`` for this process (None: re-read the environment lazily)."""
    global _current
    _current = cfg


def log_config(rank: int, cfg: Optional[RLAConfig] = None) -> None:
    if rank == 0:
        log.info((cfg or get_config()).describe())


def gpu_pg_backend() -> str:
    """Process-group backend for a GPU worker under the current config."""
    return "gloo" if get_config().pg_backend == "gloo" else "nccl"
