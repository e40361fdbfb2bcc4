import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    # Start the actor-runtime node launcher BEFORE any test touches the GPU:
    # worker processes are then forked by a process that never initialised HIP.
    try:
        from ray_lightning_accelerators_amd.runtime import launcher

        launcher.prestart()
    except Exception:  # runtime optional during early bring-up
        pass


def gpu_count() -> int:
    import torch

    return torch.cuda.device_count()


requires_gpu = pytest.mark.skipif(
    "os.environ.get('RLA_FORCE_NO_GPU') == '1'", reason="GPU disabled by env")


def pytest_runtest_setup(item):
    # debug census (RLA_DBG_THREADS=1): threads alive before the MNIST one-launch fidelity test
    import os
    if os.environ.get("RLA_DBG_THREADS") == "1" and "one_launch_grads" in item.nodeid:
        import sys
        import threading
        names = [(t.name, type(t).__name__, t.daemon) for t in threading.enumerate()]
        print(f"\n[threads before {item.nodeid}] {len(names)}: {names}", file=sys.stderr, flush=True)
