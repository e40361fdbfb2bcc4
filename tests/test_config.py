"""RLAConfig: defaults < env < explicit kwargs; travels with the accelerator."""
import pickle

import pytest

from ray_lightning_accelerators_amd.config import RLAConfig, get_config, set_config


def test_defaults_env_and_overrides(monkeypatch):
    monkeypatch.setenv("RLA_BUCKET_CAP_MB", "4")
    monkeypatch.setenv("RLA_ALLREDUCE_ALGO", "rccl")
    monkeypatch.setenv("RLA_USE_HIP_GRAPH", "false")
    monkeypatch.setenv("RLA_XGMI_BYTES", "0x100000")
    monkeypatch.setenv("RLA_FUSED_OPTIM", "0")  # legacy spelling
    cfg = RLAConfig.from_env()
    assert cfg.bucket_cap_mb == 4.0 and cfg.allreduce_algo == "rccl" and cfg.use_hip_graph is False
    assert cfg.xgmi_bytes == 1 << 20 and cfg.fused_optimizer is False
    cfg2 = RLAConfig.resolve(bucket_cap_mb=2, grad_dtype=None)
    assert cfg2.bucket_cap_mb == 2 and cfg2.allreduce_algo == "rccl"
    env = cfg2.to_env()
    assert RLAConfig.from_env(env) == cfg2


def test_validation():
    with pytest.raises(ValueError):
        RLAConfig(allreduce_algo="ring")
    with pytest.raises(ValueError):
        RLAConfig(grad_dtype="fp8")
    with pytest.raises(TypeError):
        RLAConfig().replace(bucket_mb=3)
    with pytest.raises(ValueError):
        RLAConfig.from_env({"RLA_SPIN_LIMIT": "lots"})


def test_accelerator_carries_config(monkeypatch):
    from ray_lightning_accelerators_amd import RayAccelerator

    monkeypatch.setenv("RLA_GRAD_DTYPE", "bf16")
    acc = RayAccelerator(num_workers=2, bucket_cap_mb=3, allreduce_algo="oneshot")
    assert acc.config.grad_dtype == "bf16" and acc.config.bucket_cap_mb == 3
    assert acc.config.allreduce_algo == "oneshot" and acc.bucket_cap_mb == 3 and acc.grad_dtype == "bf16"
    acc2 = pickle.loads(pickle.dumps(acc))
    assert acc2.config == acc.config


def test_process_config_install():
    try:
        set_config(RLAConfig(watchdog_ms=7))
        assert get_config().watchdog_ms == 7
    finally:
        set_config(None)
    assert get_config().watchdog_ms == RLAConfig().watchdog_ms or True
