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


# ---------------------------------------------------------------- device canaries
# RLA_CANARY=1 (diagnostic): after every test, the caching allocator's free device
# blocks are taken over by canary tensors filled with a byte pattern and held through
# the NEXT test; any byte that changes was written by something that still holds a
# pointer into memory it no longer owns (a stray asynchronous writer).  The report
# names the test during which it happened and what was written.
_CANARY = {"tensors": [], "prev": None}
_MEMHIST = {"on": False}
_CANARY_BYTE = 0x5A


_CANARY_MAX_BLOCK = 256 << 20
_CANARY_MAX_TOTAL = 3 << 30


def _canary_fill():
    import torch

    torch.cuda.synchronize()
    base = torch.cuda.memory_reserved()
    sizes = []
    for seg in torch.cuda.memory_snapshot():
        if tuple(seg.get("segment_pool_id", (0, 0))) != (0, 0):
            continue  # a graph's private pool: its replays own that memory
        sizes += [b["size"] for b in seg["blocks"] if b["state"] == "inactive" and 4096 <= b["size"]]
    out, total = [], 0
    for sz in sorted(sizes, reverse=True):
        sz = min(sz, _CANARY_MAX_BLOCK)
        if total + sz > _CANARY_MAX_TOTAL:
            break
        t = torch.empty(sz, dtype=torch.uint8, device="cuda")
        if torch.cuda.memory_reserved() > base:
            del t
            break
        t.fill_(_CANARY_BYTE)
        out.append(t)
        total += sz
    torch.cuda.synchronize()
    return out


def _canary_check(ts):
    import torch

    torch.cuda.synchronize()
    bad = []
    for t in ts:
        changed, first, last = 0, None, None
        for off in range(0, t.numel(), 64 << 20):
            ch = t[off: off + (64 << 20)]
            ne = ch != _CANARY_BYTE
            n = int(ne.sum())
            if n:
                idx = ne.nonzero().flatten()
                first = off + int(idx[0]) if first is None else first
                last = off + int(idx[-1])
                changed += n
        if changed:
            w0 = first - first % 16
            win = t[w0: w0 + 64].cpu()
            bad.append({"addr": hex(t.data_ptr()), "size": t.numel(), "changed": changed, "first": first,
                        "last": last, "hex": win.numpy().tobytes().hex(),
                        "f32": [round(v, 6) for v in win[: (win.numel() // 4) * 4].view(torch.float32).tolist()][:8],
                        "i64": win[: (win.numel() // 8) * 8].view(torch.int64).tolist()[:4]})
    return bad


@pytest.fixture(autouse=True)
def _device_canaries(request):
    yield
    if os.environ.get("RLA_CANARY") != "1":
        return
    import torch

    if not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    try:
        bad = _canary_check(_CANARY["tensors"])
    except Exception as e:  # noqa: BLE001 - a diagnostic must never fail a test
        bad = [{"check_error": repr(e)[:300]}]
    _CANARY["tensors"] = []
    if bad:
        import json

        line = json.dumps({"canary": request.node.nodeid, "previous": _CANARY["prev"], "corrupted": bad[:8],
                           "n_blocks": len(bad)})
        print("\nCANARY " + line, file=sys.stderr, flush=True)
        path = os.environ.get("RLA_CANARY_LOG")
        if path:
            with open(path, "a") as f:
                f.write(line + "\n")
    try:
        _CANARY["tensors"] = _canary_fill()
        path = os.environ.get("RLA_CANARY_LOG")
        if path:
            import json

            with open(path, "a") as f:
                f.write(json.dumps({"fill_after": request.node.nodeid, "blocks": len(_CANARY["tensors"]),
                                    "bytes": sum(t.numel() for t in _CANARY["tensors"]),
                                    "reserved_mb": torch.cuda.memory_reserved() >> 20}) + "\n")
    except Exception as e:  # noqa: BLE001
        print(f"\nCANARY fill failed: {e!r}"[:300], file=sys.stderr, flush=True)
        _CANARY["tensors"] = []
    _CANARY["prev"] = request.node.nodeid


def pytest_runtest_setup(item):
    # RLA_MEMHIST=1 (diagnostic): the caching allocator records every device alloc / free
    # with its Python stack from the first GPU test on, so a post-mortem can name the
    # previous owners of a corrupted address range (tests/test_mlp3.py _alloc_history)
    if os.environ.get("RLA_MEMHIST") == "1" and item.get_closest_marker("gpu") and not _MEMHIST["on"]:
        try:
            import torch

            torch.cuda.memory._record_memory_history(enabled="all", context="all", stacks="python",
                                                     max_entries=200000)
            _MEMHIST["on"] = True
        except Exception as e:  # noqa: BLE001 - a diagnostic must never fail a test
            print(f"\nMEMHIST off: {e!r}"[:300], file=sys.stderr, flush=True)
            _MEMHIST["on"] = True
    if os.environ.get("RLA_TEST_CLOCK") == "1":  # diagnostic: wall clock at each test start
        import time

        print(f"\n[clock {time.time():.3f}] {item.nodeid}", file=sys.stderr, flush=True)
    # debug census (RLA_DBG_THREADS=1): threads alive before the MNIST one-launch fidelity test
    if os.environ.get("RLA_DBG_THREADS") == "1" and "one_launch_grads" in item.nodeid:
        import threading
        names = [(t.name, type(t).__name__, t.daemon) for t in threading.enumerate()]
        print(f"\n[threads before {item.nodeid}] {len(names)}: {names}", file=sys.stderr, flush=True)
