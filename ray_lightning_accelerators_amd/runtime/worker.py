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
        self.parked = False  # set by a "park" request: serve() returns, the process is recycled
        self.conns = set()
        self.conns_lock = threading.Lock()

    def _park(self, conn: P.SafeConn, call_id) -> None:
        """Recycle this process (head's kill of a reusable actor): run the instance's
        ``__rla_park__`` reset (process groups, communicators, sessions), drop it,
        acknowledge, then stop serving -- every client connection is closed, so a
        stale handle sees the actor as dead, never the next tenant."""
        ok = True
        try:
            fn = getattr(self.instance, "__rla_park__", None)
            if fn is not None:
                fn()
        except BaseException:  # noqa: BLE001 - an unclean reset ends the process instead
            traceback.print_exc()
            ok = False
        self.instance = None
        try:
            conn.send({"call_id": call_id, "ok": ok})
        except Exception:
            pass
        if not ok:
            os._exit(1)
        self.parked = True
        with self.conns_lock:
            conns, self.conns = list(self.conns), set()
        for c in conns:
            try:
                c.close()
            except Exception:
                pass
        try:  # wake serve()'s accept (closing a listener does not interrupt a blocked accept)
            P.connect(self.address, self.authkey).close()
        except Exception:
            pass
        import gc

        gc.collect()  # after the ack: the killer (a trial's teardown) does not wait for it

    def _run_call(self, conn: P.SafeConn, msg: dict) -> None:
        kind = msg["kind"]
        call_id = msg["call_id"]
        try:
            args, kwargs = P.loads(msg["payload"])
            if len(msg["payload"]) > (1 << 16):
                from ..utils.timeline import mark

                mark("call_unpickled", bytes=len(msg["payload"]), method=msg.get("method"))
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
            if msg.get("kind") == "park":
                # after every call already submitted (same executor, in order)
                self.executor.submit(self._park, conn, msg.get("call_id"))
                return
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
        while not self.parked:
            try:
                c = self.listener.accept()
            except (OSError, EOFError):
                continue
            if self.parked:
                c.close()
                break
            sc = P.SafeConn(c)
            with self.conns_lock:
                self.conns.add(sc)
            threading.Thread(target=self._serve_conn, args=(sc,), daemon=True).start()
        try:
            self.listener.close()
        except Exception:
            pass
        self.executor.shutdown(wait=False)


def _warm_optimizer() -> None:
    import torch

    # the first optimizer construction imports torch._dynamo (~1 s)
    torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))])


def _warm_imports(background: bool = False) -> None:
    """``background``: report ready after the module imports and finish the
    optimizer warm-up on a thread (utils/warmup.py) -- a pooled worker becomes
    usable ~1 s sooner, which a cold Tune sweep's first trial driver waits for."""
    import torch  # noqa: F401 - the import is the point: it is what a pooled worker saves
    import torch.distributed  # noqa: F401

    # the framework's pure-Python layers are what every training worker unpickles next
    import ray_lightning_accelerators_amd.accelerators.ray_ddp  # noqa: F401
    import ray_lightning_accelerators_amd.lightning  # noqa: F401
    import ray_lightning_accelerators_amd.models.datamodules  # noqa: F401
    import ray_lightning_accelerators_amd.tune  # noqa: F401

    if background:
        from ..utils import warmup

        warmup.start(_warm_optimizer)
    else:
        _warm_optimizer()


def _warm_gpu() -> bool:
    """Pre-warmed recyclable worker: initialise HIP on this process's GPU and load
    the native kernel libraries (what the first step of a fresh worker pays)."""
    try:
        import torch

        try:  # the checkpoint writer, forked before anything touches the GPU (utilities.py)
            from ray_lightning_accelerators_amd.lightning.utilities import process_checkpoint_writer

            process_checkpoint_writer()
        except Exception:  # noqa: BLE001 - optional
            traceback.print_exc()
        if not torch.cuda.is_available():
            return False
        torch.cuda.init()
        torch.zeros(1, device="cuda").add_(1)
        from ray_lightning_accelerators_amd import ops
        from ray_lightning_accelerators_amd.parallel.comm import native_comm_module

        ops.require()
        native_comm_module()
        # first-use costs a training worker would otherwise pay inside its first fit:
        # the optimizer's device paths and a GEMM library (measured: ~1.6 s in the
        # first Tune trial's configure_optimizers / first steps, profiles/r3_tune)
        p = torch.nn.Parameter(torch.zeros(64, device="cuda"))
        opt = torch.optim.Adam([p], lr=1e-3)
        lin = torch.nn.Linear(64, 64).cuda()
        (lin(p.view(1, 64)).sum()).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        del opt, lin, p
        torch.cuda.synchronize()
        return True
    except Exception:  # noqa: BLE001 - no usable GPU here: just do not park
        traceback.print_exc()
        return False


def _wait_for_assignment(op: str = "pool_ready") -> None:
    """Block until the head assigns an actor; apply its environment
    (HIP_VISIBLE_DEVICES, actor id, ...), working directory and log file.
    ``op``: "pool_ready" (pre-started pool worker: imports done, GPU untouched) or
    "parked" (recycled / pre-warmed worker: HIP initialised on its GPU; the head
    only hands it to an actor of the same key and GPU tokens)."""
    head = P.connect(os.environ[P.ENV_HEAD], bytes.fromhex(os.environ[P.ENV_AUTH]))
    torch = sys.modules.get("torch")
    warm = bool(torch is not None and torch.cuda.is_initialized())
    head.send({"op": op, "pid": os.getpid(), "gpu_ready": warm})
    try:
        msg = head.recv()
    except (EOFError, OSError):
        os._exit(0)  # head gone: nobody will ever assign this worker
    head.close()
    if msg.get("replace"):
        # a recycled process: its environment is exactly the new actor's
        for k in list(os.environ):
            if k not in msg["env"]:
                os.environ.pop(k, None)
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
    if n and n.isdigit() and "torch" in sys.modules:
        sys.modules["torch"].set_num_threads(int(n))  # libgomp read the head's value at import


def main() -> None:
    argv = sys.argv[1:]
    extra = os.environ.get(P.ENV_SYS_PATH, "")
    for p in reversed([x for x in extra.split(os.pathsep) if x]):
        if p not in sys.path:
            sys.path.insert(0, p)
    if "--pool" in argv:
        _warm_imports(background=True)
        _wait_for_assignment("pool_ready")
    elif "--prewarm" in argv:
        from ..utils.timeline import mark

        mark("prewarm_start")
        _warm_imports()
        mark("prewarm_imports_done")
        if not _warm_gpu():
            os._exit(0)
        mark("prewarm_gpu_done")
        _wait_for_assignment("parked")
    from . import client

    while True:
        client._mark_worker()
        srv = WorkerServer()
        srv.serve()  # returns only when the head recycled this process
        _wait_for_assignment("parked")


if __name__ == "__main__":
    main()
