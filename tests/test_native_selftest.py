"""Native comm-engine self-test binaries (csrc/comm/selftest.cpp).

``build/comm_selftest`` forks W ranks that drive the xGMI one-shot / two-shot
kernels, the fusion engine thread and the DDP reducer without Python in the
loop; ``build/comm_selftest_asan`` is the same program with AddressSanitizer,
UndefinedBehaviorSanitizer and LeakSanitizer on the host code (device code is
not instrumented).  Built by ``python -m ray_lightning_accelerators_amd._build
--selftest`` / ``__graft_entry__.build()``.
"""
import os
import subprocess

import pytest

from ray_lightning_accelerators_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUPP = os.path.join(ROOT, "scripts", "sanitizers", "lsan.supp")


def _binary(sanitize):
    p = _build.selftest_path(sanitize)
    if not p.exists():
        pytest.skip(f"{p.name} not built (python -m ray_lightning_accelerators_amd._build --selftest)")
    return str(p)


def _asan_env():
    env = dict(os.environ)
    env.update(ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:protect_shadow_gap=0",
               LSAN_OPTIONS=f"suppressions={SUPP}:print_suppressions=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return env


def test_asan_build_is_instrumented():
    """CPU: the sanitizer build must report a planted heap overflow."""
    exe = _binary(True)
    env = _asan_env()
    env["ASAN_OPTIONS"] += ":detect_leaks=0"
    p = subprocess.run([exe, "canary"], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode != 0 and "heap-buffer-overflow" in p.stderr, p.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_native_selftest(world):
    p = subprocess.run([_binary(False), str(world)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and f"PASSED (world {world})" in p.stdout, (p.stdout[-3000:], p.stderr[-3000:])


@pytest.mark.gpu
def test_native_selftest_under_asan_ubsan():
    p = subprocess.run([_binary(True), "2"], capture_output=True, text=True, timeout=300, env=_asan_env())
    assert p.returncode == 0 and "PASSED (world 2)" in p.stdout, (p.stdout[-3000:], p.stderr[-3000:])
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error:" not in p.stderr, p.stderr[-3000:]
