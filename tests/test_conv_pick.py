"""Backend choice of the NHWC convolution ops (ops/conv.py) under
Trainer(deterministic=True): fixed, never timed."""
import torch

from ray_lightning_accelerators_amd.ops import conv


def test_deterministic_mode_pins_backend_without_timing(monkeypatch):
    monkeypatch.setenv("RLA_CONV1X1", "auto")
    monkeypatch.setenv("RLA_CONV_WGRAD", "auto")

    def boom():
        raise AssertionError("timed a candidate in deterministic mode")

    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        assert conv._pick("wgrad", (64, 64, 64), {"gemm": boom, "miopen": boom, "hip": boom}) == "hip"
        assert conv._pick("wgrad_kxk", (1, 64, 64, 3, 3, 1, 1), {"miopen": boom, "hip_gen": boom}) == "hip_gen"
        assert conv._pick("fwd", (64, 64, 64), {"gemm": boom, "miopen": boom}) == "gemm"
        assert conv._pick("dgrad", (64, 64, 64), {"miopen": boom}) == "miopen"
    finally:
        torch.use_deterministic_algorithms(prev)
    assert not conv._choice, "deterministic picks must not populate the timed cache"
