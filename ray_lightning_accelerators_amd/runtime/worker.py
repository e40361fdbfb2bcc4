"""Actor worker process: hosts ONE actor instance and executes its method calls.

Started by the head (``python -m ray_lightning_accelerators_amd.runtime.worker``)
with the GPU pinned through ``HIP_VISIBLE_DEVICES``/``CUDA_VISIBLE_DEVICES``.
Calls arrive on any number of client connections (the creator, plus anyone
the handle was passed to -- e.g. training workers calling the Tune queue
actor) and run in submission order on one executor thread (or a small pool
when the actor was created with ``max_concurrency > 1``).
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import traceback
from concurrent.futures import ThreadPoolExecutor

from . import protocol as P


class WorkerServer:
    def __init__(self):
        self.authkey = bytes.fromhex(os.environ[P.ENV_AUTH])
        self.session_dir = os.environ[P.ENV_SESSION_DIR]
        self.actor_id = os.environ[P.ENV_ACTOR_ID]
        self.listener, self.address = P.make_listener(self.session_dir, self.authkey, f"actor-{self.actor_id[:8]}")
        self.instance = None
        self.executor = ThreadPoolExecutor(max_workers=1)
        self.exiting = False

    def _run_call(self, conn: P.SafeConn, msg: dict) -> None:
        kind = msg["kind"]
        call_id = msg["call_id"]
        try:
            args, kwargs = P.loads(msg["payload"])
            if kind == "init":
                cls = P.loads(msg["cls"])
                conc = int(msg.get("max_concurrency", 1) or 1)
                if conc > 1:
                    self.executor = ThreadPoolExecutor(max_workers=conc)
                self.instance = cls(*args, **kwargs)
                result = None
            elif kind == "call":
                fn = getattr(self.instance, msg["method"])
                result = fn(*args, **kwargs)
            elif kind == "exec":  # run a free function (task semantics)
                fn = P.loads(msg["fn"])
                result = fn(*args, **kwargs)
            else:
                raise ValueError(f"unknown call kind {kind}")
            reply = {"call_id": call_id, "ok": True, "value": P.dumps(result)}
        except SystemExit:
            reply = {"call_id": call_id, "ok": False, "error": {"repr": "SystemExit", "tb": "", "exc": None}}
            self.exiting = True
        except BaseException as e:  # noqa: BLE001 - shipped back to the caller
            reply = {"call_id": call_id, "ok": False, "error": P.pack_exception(e)}
        try:
            conn.send(reply)
        except Exception:
            # result not picklable: report that instead
            try:
                conn.send({"call_id": call_id, "ok": False,
                           "error": {"repr": "UnpicklableResult", "tb": traceback.format_exc(), "exc": None}})
            except Exception:
                pass
        if self.exiting:
            os._exit(0)

    def _serve_conn(self, conn: P.SafeConn) -> None:
        while True:
            try:
                msg = conn.recv()
            except (EOFError, OSError):
                return
            except Exception:
                traceback.print_exc()
                return
            if msg.get("kind") == "exit":
                os._exit(0)
            if msg.get("kind") == "init":
                # construction must finish before any method runs
                self._run_call(conn, msg)
            else:
                self.executor.submit(self._run_call, conn, msg)

    def serve(self) -> None:
        head = P.connect(os.environ[P.ENV_HEAD], self.authkey)
        head.send({"op": "register", "actor_id": self.actor_id, "address": self.address, "pid": os.getpid()})
        head.recv()
        head.close()
        while True:
            try:
                c = self.listener.accept()
            except (OSError, EOFError):
                continue
            threading.Thread(target=self._serve_conn, args=(P.SafeConn(c),), daemon=True).start()


def _wait_for_assignment() -> None:
    """Pre-started pool worker: import the heavy modules now (never touching a
    GPU), then block until the head assigns an actor; apply its environment
    (HIP_VISIBLE_DEVICES, actor id, ...), working directory and log file."""
    import torch  # noqa: F401 - the import is the point: it is what a pooled worker saves
    import torch.distributed  # noqa: F401

    # the first optimizer construction imports torch._dynamo (~1 s); the framework's
    # pure-Python layers are what every training worker unpickles next (no GPU call)
    torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))])
    import ray_lightning_accelerators_amd.accelerators.ray_ddp  # noqa: F401
    import ray_lightning_accelerators_amd.lightning  # noqa: F401
    import ray_lightning_accelerators_amd.models.datamodules  # noqa: F401
    import ray_lightning_accelerators_amd.tune  # noqa: F401

    head = P.connect(os.environ[P.ENV_HEAD], bytes.fromhex(os.environ[P.ENV_AUTH]))
    head.send({"op": "pool_ready", "pid": os.getpid()})
    try:
        msg = head.recv()
    except (EOFError, OSError):
        os._exit(0)  # head gone: nobody will ever assign this worker
    head.close()
    for k in msg.get("unset", []):
        os.environ.pop(k, None)
    os.environ.update(msg.get("env") or {})
    os.chdir(msg.get("cwd") or os.getcwd())
    fd = os.open(msg["log"], os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
    sys.stdout.flush()
    sys.stderr.flush()
    os.dup2(fd, 1)
    os.dup2(fd, 2)
    os.close(fd)
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit():
        torch.set_num_threads(int(n))  # libgomp read the head's value at import


def main() -> None:
    pooled = "--pool" in sys.argv[1:]
    extra = os.environ.get(P.ENV_SYS_PATH, "")
    for p in reversed([x for x in extra.split(os.pathsep) if x]):
        if p not in sys.path:
            sys.path.insert(0, p)
    if pooled:
        _wait_for_assignment()
    from . import client

    client._mark_worker()
    WorkerServer().serve()


if __name__ == "__main__":
    main()
