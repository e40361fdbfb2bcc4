"""The example CLIs (reference examples/*.py workflows) run end to end on CPU
in ``--smoke-test`` mode (reference CI job "test_examples": .github/workflows/test.yaml)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "examples", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("name", ["ray_ddp_example", "ray_horovod_example"])
def test_example_smoke(name, tmpdir, monkeypatch):
    monkeypatch.chdir(tmpdir)
    _load(name).main(["--smoke-test"])


def test_example_tune_smoke(tmpdir, monkeypatch):
    monkeypatch.chdir(tmpdir)
    monkeypatch.setenv("TUNE_RESULTS_DIR", str(tmpdir))
    analysis = _load("ray_ddp_tune").main(["--smoke-test"])
    assert analysis.best_config is not None and analysis.best_checkpoint is not None
