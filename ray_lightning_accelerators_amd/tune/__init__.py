"""Tune-compatible hyper-parameter sweep runner + Lightning reporting callbacks.

``tune.run``/``choice``/``loguniform``/``with_parameters``/``report``/
``checkpoint_dir``/``is_session_enabled`` (the ray.tune surface used by the
reference) and ``TuneReportCallback`` /
``TuneReportCheckpointCallback`` (reference ray_lightning/tune.py).
"""
from .analysis import ExperimentAnalysis, Trial  # noqa: F401
from .callbacks import TuneCallback, TuneReportCallback, TuneReportCheckpointCallback, _TuneCheckpointCallback  # noqa: F401
from .runner import run, with_parameters  # noqa: F401
from .sample import (  # noqa: F401
    choice,
    grid_search,
    lograndint,
    loguniform,
    quniform,
    randint,
    randn,
    sample_from,
    uniform,
)
from .schedulers import ASHAScheduler, AsyncHyperBandScheduler, FIFOScheduler, TrialScheduler  # noqa: F401
from .session import checkpoint_dir, get_trial_dir, get_trial_id, is_session_enabled, report  # noqa: F401

TUNE_INSTALLED = True
