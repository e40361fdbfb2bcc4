"""Process launcher for the runtime head.

On this platform a process that has initialised the GPU must never exec()
another program (a fork+exec from it counts).  Worker processes are therefore
always forked by the head, which never touches the GPU; and the head itself is
started either directly (when the caller has not initialised HIP) or through a
tiny *fork server* started early (``prestart()``, e.g. from a test conftest
before any GPU test runs).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time
from multiprocessing.connection import Client, Listener
from typing import Optional, Tuple

ENV_LAUNCHER = "RLA_LAUNCHER_ADDRESS"
ENV_LAUNCHER_KEY = "RLA_LAUNCHER_KEY"

_server_proc: Optional[subprocess.Popen] = None


def _gpu_initialised() -> bool:
    mod = sys.modules.get("torch")
    if mod is None:
        return False
    try:
        return bool(mod.cuda.is_initialized())
    except Exception:
        return False


def _start_head_direct(session_dir: str, authkey: bytes, nodes_json: str, sys_path: str,
                       parent_pid: int) -> Tuple[str, subprocess.Popen]:
    r, w = os.pipe()
    env = dict(os.environ)
    env["RLA_AUTHKEY"] = authkey.hex()
    env["RLA_SYS_PATH"] = sys_path
    cmd = [sys.executable, "-m", "ray_lightning_accelerators_amd.runtime.head", "--session-dir", session_dir,
           "--nodes", nodes_json, "--ready-fd", str(w), "--parent-pid", str(parent_pid)]
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = os.pathsep.join([pkg_root] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p])
    log = open(os.path.join(session_dir, "head.log"), "ab")
    proc = subprocess.Popen(cmd, env=env, pass_fds=(w,), stdout=log, stderr=subprocess.STDOUT,
                            start_new_session=True)
    log.close()
    os.close(w)
    buf = b""
    deadline = time.time() + 60
    with os.fdopen(r, "rb", buffering=0) as f:
        while not buf.endswith(b"\n"):
            if time.time() > deadline:
                proc.kill()
                raise RuntimeError("runtime head did not start in 60s")
            chunk = f.read(4096)
            if not chunk:
                raise RuntimeError(f"runtime head exited (code {proc.poll()}); see {session_dir}/head.log")
            buf += chunk
    return buf.decode().strip(), proc


class _RemoteProc:
    """Popen-like stand-in for a head started by the fork server."""

    def __init__(self, pid: int):
        self.pid = pid

    def wait(self, timeout=None):
        deadline = None if timeout is None else time.time() + timeout
        while True:
            try:
                os.kill(self.pid, 0)
            except ProcessLookupError:
                return 0
            if deadline is not None and time.time() > deadline:
                raise subprocess.TimeoutExpired("head", timeout)
            time.sleep(0.05)

    def kill(self):
        try:
            os.kill(self.pid, 9)
        except ProcessLookupError:
            pass

    def poll(self):
        try:
            os.kill(self.pid, 0)
            return None
        except ProcessLookupError:
            return 0


def start_head(session_dir: str, authkey: bytes, nodes_json: str, sys_path: str):
    addr = os.environ.get(ENV_LAUNCHER)
    if addr:
        try:
            c = Client(addr, family="AF_UNIX", authkey=bytes.fromhex(os.environ[ENV_LAUNCHER_KEY]))
            c.send({"session_dir": session_dir, "authkey": authkey.hex(), "nodes": nodes_json,
                    "sys_path": sys_path, "parent_pid": os.getpid()})
            reply = c.recv()
            c.close()
            if reply.get("ok"):
                return reply["address"], _RemoteProc(reply["pid"])
        except (OSError, EOFError, KeyError):
            pass
    if _gpu_initialised():
        raise RuntimeError(
            "runtime.init() called after this process initialised the GPU and no launcher is running: "
            "call ray_lightning_accelerators_amd.runtime.launcher.prestart() (or init()) before using the GPU")
    return _start_head_direct(session_dir, authkey, nodes_json, sys_path, os.getpid())


# ----------------------------------------------------------- fork server
def _serve(address: str, key: bytes, parent_pid: int) -> None:
    lst = Listener(address, family="AF_UNIX", authkey=key)

    def watch():
        while True:
            time.sleep(1.0)
            try:
                os.kill(parent_pid, 0)
            except ProcessLookupError:
                os._exit(0)

    threading.Thread(target=watch, daemon=True).start()
    while True:
        try:
            c = lst.accept()
        except (OSError, EOFError):
            continue
        try:
            req = c.recv()
            addr, proc = _start_head_direct(req["session_dir"], bytes.fromhex(req["authkey"]), req["nodes"],
                                            req["sys_path"], int(req["parent_pid"]))
            c.send({"ok": True, "address": addr, "pid": proc.pid})
            threading.Thread(target=proc.wait, daemon=True).start()  # reap
        except Exception as e:  # noqa: BLE001
            try:
                c.send({"ok": False, "error": repr(e)})
            except OSError:
                pass
        finally:
            c.close()


def prestart() -> None:
    """Start the fork server now (before this process touches the GPU)."""
    global _server_proc
    if os.environ.get(ENV_LAUNCHER) or _gpu_initialised():
        return
    import tempfile
    import uuid

    key = os.urandom(16)
    addr = os.path.join(tempfile.gettempdir(), f"rla-launcher-{uuid.uuid4().hex[:10]}.sock")
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([pkg_root] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p])
    _server_proc = subprocess.Popen(
        [sys.executable, "-c",
         "import sys; from ray_lightning_accelerators_amd.runtime.launcher import _serve; "
         "_serve(sys.argv[1], bytes.fromhex(sys.argv[2]), int(sys.argv[3]))", addr, key.hex(), str(os.getpid())],
        env=env, start_new_session=True)
    for _ in range(200):
        if os.path.exists(addr):
            break
        time.sleep(0.02)
    os.environ[ENV_LAUNCHER] = addr
    os.environ[ENV_LAUNCHER_KEY] = key.hex()


def stop() -> None:
    global _server_proc
    if _server_proc is not None:
        _server_proc.kill()
        _server_proc = None
    os.environ.pop(ENV_LAUNCHER, None)
    os.environ.pop(ENV_LAUNCHER_KEY, None)


def dumps_nodes(nodes) -> str:
    return json.dumps(nodes)
