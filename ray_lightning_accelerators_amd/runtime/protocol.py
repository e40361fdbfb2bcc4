"""Wire helpers shared by the head, workers and clients of the actor runtime.

Frames are cloudpickle payloads over ``multiprocessing.connection`` AF_UNIX
sockets (authenticated with a per-session key).  This is control plane only:
no tensor ever moves through here on a training step.
"""
from __future__ import annotations

import os
import socket
import tempfile
import threading
import traceback
import uuid
from multiprocessing.connection import Client, Connection, Listener
from typing import Any, Optional, Tuple

import cloudpickle

ENV_HEAD = "RLA_HEAD_ADDRESS"
ENV_AUTH = "RLA_AUTHKEY"
ENV_SESSION_DIR = "RLA_SESSION_DIR"
ENV_NODE_IP = "RLA_NODE_IP"
ENV_NODE_ADDR = "RLA_NODE_ADDR"
ENV_ACTOR_ID = "RLA_ACTOR_ID"
ENV_SYS_PATH = "RLA_SYS_PATH"


def new_id() -> str:
    return uuid.uuid4().hex


def dumps(obj: Any) -> bytes:
    return cloudpickle.dumps(obj)


def loads(b: bytes) -> Any:
    return cloudpickle.loads(b)


class SafeConn:
    """A Connection with a send lock (many threads may submit on one socket)."""

    def __init__(self, conn: Connection):
        self.conn = conn
        self._lock = threading.Lock()

    def send(self, obj: Any) -> None:
        data = dumps(obj)
        with self._lock:
            self.conn.send_bytes(data)

    def recv(self) -> Any:
        return loads(self.conn.recv_bytes())

    def close(self) -> None:
        try:
            self.conn.close()
        except OSError:
            pass


def make_listener(session_dir: str, authkey: bytes, prefix: str) -> Tuple[Listener, str]:
    path = os.path.join(session_dir, f"{prefix}-{uuid.uuid4().hex[:12]}.sock")
    lst = Listener(address=path, family="AF_UNIX", authkey=authkey)
    return lst, path


def connect(address: str, authkey: bytes) -> SafeConn:
    return SafeConn(Client(address=address, family="AF_UNIX", authkey=authkey))


def new_session_dir() -> str:
    base = os.environ.get("RLA_TMPDIR") or tempfile.gettempdir()
    return tempfile.mkdtemp(prefix="rla-session-", dir=base)


def host_ip_address() -> str:
    """This host's outbound IP (no per-worker override)."""
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
        finally:
            s.close()
    except OSError:
        return "127.0.0.1"


def reachable_address(ip: str, index: int) -> str:
    """Address at which sockets of node ``ip`` (the ``index``-th node of the session)
    are reachable: the IP of a real node (this host's, or a loopback address), a
    distinct loopback alias (127.0.0.<index + 1>) for a simulated node -- every
    simulated node is a process group on this host, and Linux routes all of
    127/8 to loopback, so per-node rendezvous addresses stay distinguishable."""
    if ip.startswith("127.") or ip in ("localhost", host_ip_address()):
        return ip
    return f"127.0.0.{index % 254 + 1}"


def node_address() -> str:
    """Reachable address of this process's node (see :func:`reachable_address`)."""
    return os.environ.get(ENV_NODE_ADDR) or node_ip_address()


def node_ip_address() -> str:
    """This process's node IP (overridable per worker for multi-node simulation)."""
    return os.environ.get(ENV_NODE_IP) or host_ip_address()


class RemoteError(Exception):
    """An exception raised inside an actor method, re-raised at ``get``."""

    def __init__(self, cause_repr: str, tb: str, cause: Optional[BaseException] = None):
        super().__init__(f"{cause_repr}\n\nRemote traceback:\n{tb}")
        self.cause = cause
        self.remote_traceback = tb


class ActorDiedError(RuntimeError):
    pass


class GetTimeoutError(TimeoutError):
    pass


def pack_exception(e: BaseException) -> dict:
    tb = traceback.format_exc()
    try:
        payload = dumps(e)
    except Exception:  # unpicklable exception
        payload = None
    return {"repr": repr(e), "tb": tb, "exc": payload}


def unpack_exception(d: dict) -> BaseException:
    """RemoteError that is ALSO an instance of the original exception type
    (``except ValueError`` keeps working across the process boundary)."""
    cause = None
    if d.get("exc") is not None:
        try:
            cause = loads(d["exc"])
        except Exception:
            cause = None
    if isinstance(cause, Exception) and not isinstance(cause, RemoteError):
        try:
            cls = type(f"RemoteError[{type(cause).__name__}]", (RemoteError, type(cause)), {})
            err = cls.__new__(cls)
            RemoteError.__init__(err, d["repr"], d["tb"], cause)
            return err
        except TypeError:
            pass
    return RemoteError(d["repr"], d["tb"], cause)
