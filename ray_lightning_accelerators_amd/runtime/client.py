"""Client side of the actor runtime (used by the driver and by every worker).

Public surface mirrors the subset of Ray the reference and its tests use
(SURVEY.md §2.9): ``init/shutdown/is_initialized``, ``remote`` (actor classes
with ``.options(num_cpus=, num_gpus=, resources=, name=, max_concurrency=)``
and remote functions), ``get/put/wait/kill``, ``actors()``,
``available_resources()/cluster_resources()``, ``get_gpu_ids()``,
``get_node_ip_address()``.
"""
from __future__ import annotations

import atexit
import inspect
import itertools
import os
import shutil
import subprocess
import sys
import threading
import time
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutTimeout
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

from . import protocol as P

_IS_WORKER = False


def _mark_worker() -> None:
    global _IS_WORKER
    _IS_WORKER = True


# --------------------------------------------------------------------- state
class _Runtime:
    def __init__(self, head_address: str, authkey: bytes, session_dir: str, owns_head: bool,
                 head_proc: Optional[subprocess.Popen] = None):
        self.head_address = head_address
        self.authkey = authkey
        self.session_dir = session_dir
        self.owns_head = owns_head
        self.head_proc = head_proc
        self._head = P.connect(head_address, authkey)
        self._head_lock = threading.Lock()
        self._conns: Dict[str, "_ActorConn"] = {}
        self._conns_lock = threading.Lock()
        self.obj_dir = os.path.join(session_dir, "objects")
        os.makedirs(self.obj_dir, exist_ok=True)

    def head_call(self, msg: dict) -> dict:
        with self._head_lock:
            self._head.send(msg)
            return self._head.recv()

    def head_call_new_conn(self, msg: dict) -> dict:
        # long-blocking requests (actor creation) get their own connection
        c = P.connect(self.head_address, self.authkey)
        try:
            c.send(msg)
            return c.recv()
        finally:
            c.close()

    def conn_for(self, address: str) -> "_ActorConn":
        with self._conns_lock:
            c = self._conns.get(address)
            if c is None or c.closed:
                c = _ActorConn(address, self.authkey)
                self._conns[address] = c
            return c

    def close(self) -> None:
        with self._conns_lock:
            for c in self._conns.values():
                c.close()
            self._conns.clear()
        if self.owns_head:
            try:
                self.head_call({"op": "shutdown"})
            except Exception:
                pass
            if self.head_proc is not None:
                try:
                    self.head_proc.wait(timeout=10)
                except Exception:
                    self.head_proc.kill()
            shutil.rmtree(self.session_dir, ignore_errors=True)
        self._head.close()


_rt: Optional[_Runtime] = None
_rt_lock = threading.RLock()
_call_ids = itertools.count(1)


def _runtime() -> _Runtime:
    global _rt
    with _rt_lock:
        if _rt is None:
            if os.environ.get(P.ENV_HEAD):
                _connect_existing()
            else:
                init()
        return _rt


def _connect_existing() -> None:
    global _rt
    _rt = _Runtime(os.environ[P.ENV_HEAD], bytes.fromhex(os.environ[P.ENV_AUTH]),
                   os.environ[P.ENV_SESSION_DIR], owns_head=False)


# ------------------------------------------------------------- connections
class _ActorConn:
    """One socket to one actor; a reader thread resolves call futures."""

    def __init__(self, address: str, authkey: bytes):
        self.address = address
        self.conn = P.connect(address, authkey)
        self.pending: Dict[int, Future] = {}
        self.lock = threading.Lock()
        self.closed = False
        self.reader = threading.Thread(target=self._read, daemon=True)
        self.reader.start()

    def submit(self, msg: dict) -> Future:
        fut: Future = Future()
        call_id = next(_call_ids)
        msg["call_id"] = call_id
        with self.lock:
            if self.closed:
                fut.set_exception(P.ActorDiedError(f"actor at {self.address} is dead"))
                return fut
            self.pending[call_id] = fut
        try:
            self.conn.send(msg)
        except (OSError, EOFError, BrokenPipeError) as e:
            self._fail_all(P.ActorDiedError(f"actor connection lost: {e!r}"))
        return fut

    def _read(self) -> None:
        while True:
            try:
                msg = self.conn.recv()
            except (EOFError, OSError, ConnectionResetError):
                self._fail_all(P.ActorDiedError(f"the actor at {self.address} died unexpectedly"))
                return
            with self.lock:
                fut = self.pending.pop(msg["call_id"], None)
            if fut is None:
                continue
            if msg["ok"]:
                try:
                    fut.set_result(P.loads(msg["value"]))
                except Exception as e:  # noqa: BLE001
                    fut.set_exception(e)
            else:
                fut.set_exception(P.unpack_exception(msg["error"]))

    def _fail_all(self, exc: BaseException) -> None:
        with self.lock:
            self.closed = True
            pend, self.pending = self.pending, {}
        for f in pend.values():
            if not f.done():
                f.set_exception(exc)

    def close(self) -> None:
        self._fail_all(P.ActorDiedError("connection closed"))
        self.conn.close()


# ------------------------------------------------------------- object refs
_MISSING = object()
_MARK_BYTES = 1 << 16  # timeline marks for payloads at least this large


def _mark(event: str, **fields) -> None:
    from ..utils.timeline import mark

    mark(event, **fields)


class ObjectRef:
    """Future-like handle to a value (a remote call result or a ``put``).

    Pickling a ref (passing it *nested* inside another argument) spills the
    value to a file in the session's object directory (shared memory when the
    session lives under /dev/shm) and the receiver loads it on ``get``.
    """

    def __init__(self, fut: Optional[Future] = None, value: Any = _MISSING, path: Optional[str] = None,
                 ref_id: Optional[str] = None):
        self.id = ref_id or P.new_id()
        self._fut = fut
        self._value = value
        self._path = path

    def _resolve(self, timeout: Optional[float] = None) -> Any:
        if self._value is not _MISSING:
            return self._value
        if self._fut is not None:
            try:
                self._value = self._fut.result(timeout=timeout)
            except FutTimeout:
                raise P.GetTimeoutError(f"get() timed out after {timeout}s")
            return self._value
        if self._path is not None:
            with open(self._path, "rb") as f:
                self._value = P.loads(f.read())
            return self._value
        raise RuntimeError("empty ObjectRef")

    def done(self) -> bool:
        if self._value is not _MISSING or self._path is not None:
            return True
        return self._fut is not None and self._fut.done()

    def future(self) -> Future:
        if self._fut is not None:
            return self._fut
        f: Future = Future()
        try:
            f.set_result(self._resolve())
        except BaseException as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def __reduce__(self):
        if self._path is None:
            value = self._resolve()
            path = os.path.join(_runtime().obj_dir, self.id)
            with open(path + ".tmp", "wb") as f:
                f.write(P.dumps(value))
            os.replace(path + ".tmp", path)
            self._path = path
        return (_ref_from_path, (self._path, self.id))

    def __repr__(self) -> str:
        return f"ObjectRef({self.id[:12]})"


def _ref_from_path(path: str, ref_id: str) -> ObjectRef:
    return ObjectRef(None, _MISSING, path, ref_id)


def _deref_args(args: Sequence[Any], kwargs: Dict[str, Any]) -> Tuple[tuple, dict]:
    """Ray semantics: top-level ObjectRef arguments are resolved before the call."""
    args = tuple(a._resolve() if isinstance(a, ObjectRef) else a for a in args)
    kwargs = {k: (v._resolve() if isinstance(v, ObjectRef) else v) for k, v in kwargs.items()}
    return args, kwargs


# ------------------------------------------------------------------ actors
class ActorMethod:
    def __init__(self, handle: "ActorHandle", name: str):
        self._handle = handle
        self._name = name

    def remote(self, *args, **kwargs) -> ObjectRef:
        return self._handle._submit({"kind": "call", "method": self._name}, args, kwargs)

    def options(self, **_kw) -> "ActorMethod":
        return self

    def __call__(self, *a, **k):
        raise TypeError(f"Actor methods cannot be called directly; use {self._name}.remote()")


class ActorHandle:
    def __init__(self, actor_id: Optional[str], address_fut: Future, meta: Optional[dict] = None):
        self._actor_id = actor_id
        self._address_fut = address_fut
        self._meta = meta or {}
        self._init_ref: Optional[ObjectRef] = None

    @property
    def _actor_id_hex(self) -> Optional[str]:
        if self._actor_id is None and self._address_fut.done() and not self._address_fut.exception():
            self._actor_id = self._address_fut.result()["actor_id"]
        return self._actor_id

    def _info(self) -> dict:
        return self._address_fut.result()

    def _submit(self, msg: dict, args, kwargs) -> ObjectRef:
        args, kwargs = _deref_args(args, kwargs)
        payload = P.dumps((args, kwargs))
        if len(payload) > _MARK_BYTES:
            _mark("submit_pickled", bytes=len(payload), method=msg.get("method"))
        out: Future = Future()

        def go(f_addr: Future):
            try:
                info = f_addr.result()
                conn = _runtime().conn_for(info["address"])
                m = dict(msg)
                m["payload"] = payload
                inner = conn.submit(m)
                inner.add_done_callback(lambda f: _chain(f, out))
            except BaseException as e:  # noqa: BLE001
                if not out.done():
                    out.set_exception(e)

        if self._address_fut.done():
            go(self._address_fut)
        else:
            self._address_fut.add_done_callback(go)
        return ObjectRef(out)

    def __getattr__(self, name: str) -> ActorMethod:
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)
        return ActorMethod(self, name)

    def __reduce__(self):
        info = self._address_fut.result()
        return (_rebuild_handle, (info, self._meta))

    def __repr__(self) -> str:
        return f"ActorHandle({self._meta.get('class_name', '?')}, {str(self._actor_id_hex)[:8]})"


def _rebuild_handle(info: dict, meta: dict) -> ActorHandle:
    f: Future = Future()
    f.set_result(info)
    return ActorHandle(info["actor_id"], f, meta)


def _chain(src: Future, dst: Future) -> None:
    if dst.done():
        return
    if src.exception() is not None:
        dst.set_exception(src.exception())
    else:
        dst.set_result(src.result())


def _resources_from(opts: dict, default_cpus: float) -> Dict[str, float]:
    res = {"CPU": float(opts.get("num_cpus", default_cpus) or 0)}
    ng = opts.get("num_gpus", 0) or 0
    if ng:
        res["GPU"] = float(ng)
    for k, v in (opts.get("resources") or {}).items():
        res[k] = float(v)
    return res


class ActorClass:
    def __init__(self, cls: type, options: Optional[dict] = None):
        self._cls = cls
        self._options = dict(options or {})
        self.__name__ = getattr(cls, "__name__", "Actor")
        self.__doc__ = cls.__doc__

    def options(self, **kw) -> "ActorClass":
        o = dict(self._options)
        o.update(kw)
        return ActorClass(self._cls, o)

    def remote(self, *args, **kwargs) -> ActorHandle:
        rt = _runtime()
        opts = self._options
        res = _resources_from(opts, default_cpus=1)
        addr_fut: Future = Future()
        meta = {"class_name": self._cls.__name__, "resources": res}
        create = {
            "op": "create_actor", "resources": res, "name": opts.get("name"),
            "class_name": self._cls.__name__, "node_ip": opts.get("_node_ip"),
            "env": opts.get("runtime_env_vars") or {},
            "sys_path": os.pathsep.join(p for p in sys.path if p),
            "cwd": os.getcwd(), "timeout": float(opts.get("_creation_timeout", 3600)),
            "owner": os.environ.get(P.ENV_ACTOR_ID),
            # recyclable worker: a kill parks the process (HIP context, loaded kernels,
            # imports kept) for the next actor with the same key, node and GPUs
            "reuse": opts.get("_reuse"),
        }
        cls_payload = P.dumps(self._cls)
        init_payload = P.dumps(_deref_args(args, kwargs))
        handle = ActorHandle(None, addr_fut, meta)

        def create_actor():
            from ..utils.timeline import mark

            try:
                mark("actor_create", cls=self._cls.__name__)
                reply = rt.head_call_new_conn(create)
                if not reply.get("ok"):
                    raise RuntimeError(f"actor creation failed: {reply.get('error')}\n{reply.get('log', '')}")
                mark("actor_registered", cls=self._cls.__name__, actor_pid=reply.get("pid"))
                conn = rt.conn_for(reply["address"])
                init = conn.submit({"kind": "init", "cls": cls_payload, "payload": init_payload,
                                    "max_concurrency": opts.get("max_concurrency", 1)})
                init.result()  # constructor errors surface on every later call
                mark("actor_ready", cls=self._cls.__name__)
                addr_fut.set_result(reply)
            except BaseException as e:  # noqa: BLE001
                addr_fut.set_exception(e)

        threading.Thread(target=create_actor, daemon=True).start()
        return handle

    def __call__(self, *a, **k):
        raise TypeError(f"Actor class {self.__name__} cannot be instantiated directly; use .remote()")


class RemoteFunction:
    """``@remote`` function: each call runs in a fresh worker process (task)."""

    def __init__(self, fn, options: Optional[dict] = None):
        self._fn = fn
        self._options = dict(options or {})
        self.__name__ = getattr(fn, "__name__", "task")

    def options(self, **kw) -> "RemoteFunction":
        o = dict(self._options)
        o.update(kw)
        return RemoteFunction(self._fn, o)

    def remote(self, *args, **kwargs) -> ObjectRef:
        runner = ActorClass(_TaskRunner, self._options).remote()
        fn_payload = P.dumps(self._fn)
        ref = runner._submit({"kind": "exec", "fn": fn_payload}, args, kwargs)

        def cleanup(_f):
            try:
                kill(runner)
            except Exception:
                pass

        ref._fut.add_done_callback(cleanup)
        return ref

    def __call__(self, *a, **k):
        return self._fn(*a, **k)


class _TaskRunner:
    pass


def remote(*args, **kwargs):
    """Decorator: ``@remote`` / ``@remote(num_cpus=..., num_gpus=...)``."""
    def wrap(obj, opts):
        if inspect.isclass(obj):
            return ActorClass(obj, opts)
        return RemoteFunction(obj, opts)

    if len(args) == 1 and not kwargs and (inspect.isclass(args[0]) or callable(args[0])):
        return wrap(args[0], {})
    return lambda obj: wrap(obj, kwargs)


# ------------------------------------------------------------- top-level API
def _node_spec(num_cpus, num_gpus, resources) -> List[dict]:
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if num_gpus is None:
        try:
            import torch

            num_gpus = torch.cuda.device_count()  # does not initialise HIP on this image
        except Exception:
            num_gpus = 0
    tokens = [t for t in vis.split(",") if t] if vis else [str(i) for i in range(num_gpus)]
    if len(tokens) < num_gpus:
        tokens += [str(i) for i in range(len(tokens), num_gpus)]
    return [{"ip": P.node_ip_address(), "num_cpus": float(num_cpus if num_cpus is not None else os.cpu_count()),
             "num_gpus": int(num_gpus), "gpu_ids": tokens[:num_gpus], "resources": resources or {}}]


def init(num_cpus: Optional[float] = None, num_gpus: Optional[int] = None, address: Optional[str] = None,
         resources: Optional[Dict[str, float]] = None, ignore_reinit_error: bool = False,
         _nodes: Optional[List[dict]] = None, **_ignored) -> dict:
    """Start (or connect to) a runtime session.

    ``address="auto"`` connects to the session in ``RLA_HEAD_ADDRESS``.
    ``_nodes`` simulates a multi-node cluster: a list of
    ``{"ip", "num_cpus", "num_gpus", "gpu_ids"}`` dicts (node-IP override for
    local-rank / multi-node tests).
    """
    global _rt
    import json

    with _rt_lock:
        if _rt is not None:
            if ignore_reinit_error or _IS_WORKER:
                return {"session_dir": _rt.session_dir}
            raise RuntimeError("runtime already initialised; call shutdown() first")
        if address not in (None, "local") or (_IS_WORKER and os.environ.get(P.ENV_HEAD)):
            if not os.environ.get(P.ENV_HEAD):
                raise ConnectionError("address='auto' but no running session (RLA_HEAD_ADDRESS unset)")
            _connect_existing()
            return {"session_dir": _rt.session_dir, "head": _rt.head_address}
        nodes = _nodes or _node_spec(num_cpus, num_gpus, resources)
        session_dir = P.new_session_dir()
        authkey = os.urandom(16)
        from . import launcher

        address_, proc = launcher.start_head(session_dir, authkey, json.dumps(nodes),
                                             os.pathsep.join(p for p in sys.path if p))
        _rt = _Runtime(address_, authkey, session_dir, owns_head=True, head_proc=proc)
        # children of this process (nested actors) find the session through env
        os.environ[P.ENV_HEAD] = address_
        os.environ[P.ENV_AUTH] = authkey.hex()
        os.environ[P.ENV_SESSION_DIR] = session_dir
        return {"session_dir": session_dir, "head": address_, "nodes": nodes}


def is_initialized() -> bool:
    return _rt is not None or bool(os.environ.get(P.ENV_HEAD) and _IS_WORKER)


def shutdown() -> None:
    global _rt
    with _rt_lock:
        if _rt is None:
            return
        rt, _rt = _rt, None
        if rt.owns_head:
            for k in (P.ENV_HEAD, P.ENV_AUTH, P.ENV_SESSION_DIR):
                os.environ.pop(k, None)
        rt.close()


atexit.register(shutdown)


def put(value: Any) -> ObjectRef:
    return ObjectRef(value=value)


def get(refs: Union[ObjectRef, Sequence[ObjectRef]], timeout: Optional[float] = None):
    if isinstance(refs, ObjectRef):
        return refs._resolve(timeout)
    if isinstance(refs, (list, tuple)):
        deadline = None if timeout is None else time.time() + timeout
        out = []
        for r in refs:
            rem = None if deadline is None else max(0.0, deadline - time.time())
            out.append(r._resolve(rem) if isinstance(r, ObjectRef) else r)
        return out
    raise TypeError(f"get() expects ObjectRef(s), got {type(refs)}")


def wait(refs: Sequence[ObjectRef], num_returns: int = 1, timeout: Optional[float] = None,
         fetch_local: bool = True) -> Tuple[List[ObjectRef], List[ObjectRef]]:
    """Return (ready, not_ready) once ``num_returns`` refs are done or ``timeout`` passes."""
    refs = list(refs)
    num_returns = min(num_returns, len(refs))
    deadline = None if timeout is None else time.time() + timeout
    cond = threading.Condition()
    for r in refs:
        if not r.done() and r._fut is not None:
            r._fut.add_done_callback(lambda _f: _notify(cond))
    with cond:
        while True:
            ready = [r for r in refs if r.done()]
            if len(ready) >= num_returns:
                break
            if deadline is not None:
                rem = deadline - time.time()
                if rem <= 0:
                    break
                cond.wait(timeout=min(rem, 0.5))
            else:
                cond.wait(timeout=0.5)
    ready_ids = {id(r) for r in ready[:max(num_returns, 0)] } if len(ready) >= num_returns else {id(r) for r in ready}
    ready_list = [r for r in refs if id(r) in ready_ids]
    return ready_list, [r for r in refs if id(r) not in ready_ids]


def _notify(cond: threading.Condition) -> None:
    with cond:
        cond.notify_all()


def kill(actor: ActorHandle, no_restart: bool = True) -> None:
    try:
        info = actor._address_fut.result(timeout=60)
    except BaseException:  # noqa: BLE001 - creation failed: nothing to kill
        return
    rt = _runtime()
    rt.head_call({"op": "kill", "actor_id": info["actor_id"], "cause": "killed via kill()"})
    with rt._conns_lock:
        c = rt._conns.pop(info["address"], None)
    if c is not None:
        c.close()


def prewarm_gpu_workers(key: str) -> dict:
    """Ask the head to start one recyclable worker per free GPU (key ``key``) that
    initialises HIP and loads the native kernels in the background, so the first
    actor created with ``.options(_reuse=key, num_gpus=1)`` skips that start-up
    (Tune sweeps of short trials; idempotent)."""
    return _runtime().head_call({"op": "prewarm", "key": key})


def actors(actor_id: Optional[str] = None) -> Dict[str, dict]:
    table = _runtime().head_call({"op": "actors"})["actors"]
    if actor_id is not None:
        return table.get(actor_id, {})
    return table


def cluster_resources() -> Dict[str, float]:
    return _runtime().head_call({"op": "resources"})["total"]


def available_resources() -> Dict[str, float]:
    return _runtime().head_call({"op": "resources"})["available"]


def nodes() -> List[dict]:
    r = _runtime().head_call({"op": "resources"})
    return [{"NodeManagerAddress": n["ip"], "Resources": n["total"], "Alive": True} for n in r["nodes"]]


def get_gpu_ids() -> List[int]:
    ids = os.environ.get("RLA_GPU_IDS", "")
    out = []
    for t in ids.split(","):
        if t.strip():
            try:
                out.append(int(t))
            except ValueError:
                out.append(t)  # non-integer device tokens (e.g. UUIDs)
    return out


def get_node_ip_address() -> str:
    return P.node_ip_address()


def get_node_address() -> str:
    """Where this node's sockets are reachable (rendezvous servers): the node IP
    of a real node, a loopback alias of a simulated one."""
    return P.node_address()


def get_actor_id() -> Optional[str]:
    return os.environ.get(P.ENV_ACTOR_ID)
