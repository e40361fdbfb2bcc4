"""Reference import path ``ray_lightning.tune`` (TuneReportCallback, TuneReportCheckpointCallback)."""
from ray_lightning_accelerators_amd.tune import (  # noqa: F401
    TUNE_INSTALLED,
    TuneCallback,
    TuneReportCallback,
    TuneReportCheckpointCallback,
    _TuneCheckpointCallback,
    is_session_enabled,
)
