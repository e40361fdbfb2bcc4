"""Node daemon ("head") of the actor runtime -- the stand-in for Ray's GCS + raylet.

Responsibilities (reference call sites in SURVEY.md §2.2 U17):
  * resource accounting per (possibly simulated) node: CPUs, GPUs (with GPU
    ids), custom resources; actors wait until their request fits;
  * spawning worker processes with ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
    set to the allocated GPU (one whole GPU per training worker, reference
    ray_ddp.py:94-96) and ``RLA_NODE_IP`` set to the node's address;
  * the actor table (ALIVE / DEAD) behind ``runtime.actors()``;
  * killing actors and noticing workers that die (fail-fast);
  * a pool of PRE-STARTED worker processes (``RLA_WORKER_POOL``, default half
    the CPUs, 2..8):
    interpreters that already imported torch but never touched a GPU wait for
    an actor assignment (env incl. HIP_VISIBLE_DEVICES, cwd, log file), so an
    actor starts in milliseconds instead of paying interpreter + torch import
    (~2 s) -- the dominant cost of short Tune trials (Ray keeps a worker pool
    for the same reason).

The head never imports torch and never touches a GPU, so it can fork workers
safely even when the driver process has already initialised HIP.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

from . import protocol as P


class Node:
    def __init__(self, ip: str, num_cpus: float, num_gpus: int, gpu_ids: List[str], resources: Dict[str, float],
                 address: str = ""):
        self.ip = ip
        # where a socket on this node is reachable from the other nodes (rendezvous
        # servers bind on the node's worker 0): the IP itself for a real node, a
        # loopback alias for a simulated one (every simulated node is this host)
        self.address = address or ip
        self.total = {"CPU": float(num_cpus), "GPU": float(num_gpus), **{k: float(v) for k, v in resources.items()}}
        self.avail = dict(self.total)
        self.free_gpus = list(gpu_ids)  # visible-device tokens in allocation order

    def fits(self, req: Dict[str, float]) -> bool:
        return all(self.avail.get(k, 0.0) + 1e-9 >= v for k, v in req.items() if v > 0)

    def take(self, req: Dict[str, float]) -> List[str]:
        for k, v in req.items():
            if v > 0:
                self.avail[k] = self.avail.get(k, 0.0) - v
        n = int(round(req.get("GPU", 0)))
        ids, self.free_gpus = self.free_gpus[:n], self.free_gpus[n:]
        return ids

    def give(self, req: Dict[str, float], gpu_ids: List[str]) -> None:
        for k, v in req.items():
            if v > 0:
                self.avail[k] = self.avail.get(k, 0.0) + v
        # keep GPU hand-out order stable (lowest id first), as Ray does per node
        self.free_gpus = sorted(self.free_gpus + list(gpu_ids), key=lambda s: (len(s), s))


class ActorRecord:
    def __init__(self, actor_id: str, name: Optional[str], req: Dict[str, float], node: Node, gpu_ids: List[str]):
        self.actor_id = actor_id
        self.name = name
        self.req = req
        self.node = node
        self.gpu_ids = gpu_ids
        self.state = "PENDING_CREATION"
        self.address: Optional[str] = None
        self.proc: Optional[subprocess.Popen] = None
        self.pid: Optional[int] = None
        self.registered = threading.Event()
        self.death_cause: Optional[str] = None
        self.class_name = ""
        self.owner: Optional[str] = None
        self.reuse: Optional[str] = None  # recyclable worker key (see Head._park)


class Head:
    def __init__(self, session_dir: str, authkey: bytes, nodes: List[Node], sys_path: str, log_dir: str):
        self.session_dir = session_dir
        self.authkey = authkey
        self.nodes = nodes
        self.sys_path = sys_path
        self.log_dir = log_dir
        self.lock = threading.Condition()
        self.actors: Dict[str, ActorRecord] = {}
        self.listener, self.address = P.make_listener(session_dir, authkey, "head")
        self.stopping = False
        # pre-started workers: pid -> Popen while starting, then (Popen, conn) when ready
        # default: half the cluster's CPUs, 2..8 (a Tune trial consumes ~3 processes:
        # trial, training worker(s), report queue)
        cpus = int(sum(n.total.get("CPU", 0) for n in nodes))
        default_pool = min(8, max(2, cpus // 2))
        self.pool_target = max(0, int(os.environ.get("RLA_WORKER_POOL", str(default_pool))))
        self.pool_starting: Dict[int, subprocess.Popen] = {}
        self.pool_ready: List = []
        self.pool_lock = threading.Lock()
        self.pool_cond = threading.Condition(self.pool_lock)  # notified when a worker parks
        # recycled workers (actors created with a reuse key): a kill parks the process
        # instead of ending it -- HIP context, loaded kernel objects and imports stay
        # -- and the next actor with the same key, node and GPU tokens takes it over.
        # parking: pid -> (Popen, key, node, gpu_ids) until the worker reports back;
        # parked: [(Popen, conn, key, node, gpu_ids)] waiting for an assignment
        self.parking: Dict[int, tuple] = {}
        self.parked: List[tuple] = []
        self.prewarming: set = set()  # pids of pre-warming workers (in `parking` until warm)
        self.prewarmed: set = set()  # (key, node ip, gpu token) already started

    # ------------------------------------------------------------ worker pool
    def _pool_env(self) -> Dict[str, str]:
        env = dict(os.environ)
        env[P.ENV_HEAD] = self.address
        env[P.ENV_AUTH] = self.authkey.hex()
        env[P.ENV_SESSION_DIR] = self.session_dir
        env[P.ENV_SYS_PATH] = self.sys_path
        env["PYTHONUNBUFFERED"] = "1"
        env.pop(P.ENV_ACTOR_ID, None)
        return env

    def refill_pool(self) -> None:
        if self.stopping:
            return
        with self.pool_lock:
            missing = self.pool_target - len(self.pool_ready) - len(self.pool_starting)
            for _ in range(max(0, missing)):
                log = open(os.path.join(self.log_dir, "pool.log"), "ab")
                proc = subprocess.Popen([sys.executable, "-m", "ray_lightning_accelerators_amd.runtime.worker", "--pool"],
                                        env=self._pool_env(), stdout=log, stderr=subprocess.STDOUT,
                                        start_new_session=True)
                log.close()
                self.pool_starting[proc.pid] = proc

    def _take_pooled(self):
        """An idle pre-started worker (its Popen and the connection it waits on), or None."""
        with self.pool_lock:
            while self.pool_ready:
                proc, conn = self.pool_ready.pop(0)
                if proc.poll() is None:
                    return proc, conn
        return None

    @staticmethod
    def _poolable(msg: dict) -> bool:
        # interpreter-start settings cannot be applied to a running process
        env = msg.get("env") or {}
        return msg.get("capture_output", True) and not any(
            k.startswith(("PYTHON", "LD_", "MALLOC")) for k in env)

    # ---------------------------------------------------------- scheduling
    def _place(self, req: Dict[str, float], node_ip: Optional[str]) -> Optional[Node]:
        for n in self.nodes:
            if node_ip is not None and n.ip != node_ip:
                continue
            if n.fits(req):
                return n
        return None

    def _feasible(self, req: Dict[str, float], node_ip: Optional[str]) -> bool:
        for n in self.nodes:
            if node_ip is not None and n.ip != node_ip:
                continue
            if all(n.total.get(k, 0.0) + 1e-9 >= v for k, v in req.items() if v > 0):
                return True
        return False

    def create_actor(self, msg: dict) -> dict:
        req = {k: float(v) for k, v in msg["resources"].items() if v}
        node_ip = msg.get("node_ip")
        if not self._feasible(req, node_ip):
            return {"ok": False, "error": f"infeasible resource request {req} (cluster: "
                                         f"{[n.total for n in self.nodes]})"}
        actor_id = P.new_id()
        deadline = time.time() + float(msg.get("timeout", 3600))
        with self.lock:
            while True:
                node = self._place(req, node_ip)
                if node is not None:
                    gpu_ids = node.take(req)
                    break
                if time.time() > deadline:
                    return {"ok": False, "error": f"timed out waiting for resources {req}"}
                self.lock.wait(timeout=0.5)
            rec = ActorRecord(actor_id, msg.get("name"), req, node, gpu_ids)
            rec.class_name = msg.get("class_name", "")
            rec.owner = msg.get("owner")
            rec.reuse = msg.get("reuse") or None
            self.actors[actor_id] = rec
        env = dict(os.environ)
        env.update(msg.get("env") or {})
        env[P.ENV_HEAD] = self.address
        env[P.ENV_AUTH] = self.authkey.hex()
        env[P.ENV_SESSION_DIR] = self.session_dir
        env[P.ENV_NODE_IP] = node.ip
        env[P.ENV_NODE_ADDR] = node.address
        env[P.ENV_ACTOR_ID] = actor_id
        env[P.ENV_SYS_PATH] = msg.get("sys_path") or self.sys_path
        if "GPU" in req:
            vis = ",".join(gpu_ids)
            env["HIP_VISIBLE_DEVICES"] = vis
            env["CUDA_VISIBLE_DEVICES"] = vis
            env.pop("ROCR_VISIBLE_DEVICES", None) if msg.get("reset_rocr") else None
        elif msg.get("hide_gpus", True):
            env["HIP_VISIBLE_DEVICES"] = ""
            env["CUDA_VISIBLE_DEVICES"] = ""
        env["RLA_GPU_IDS"] = ",".join(gpu_ids)
        env["PYTHONUNBUFFERED"] = "1"
        # Ray's contract: an actor's intra-op thread pools are sized to the CPUs it
        # reserved (OMP_NUM_THREADS = num_cpus, at least 1) unless the caller chose;
        # N workers x all-core OpenMP pools oversubscribe the node (measured: 2 MNIST
        # workers on 8 CPUs ran 64 ms/step instead of ~2 ms)
        if "OMP_NUM_THREADS" not in (msg.get("env") or {}):
            env["OMP_NUM_THREADS"] = str(max(1, int(req.get("CPU", 1) or 1)))
        log_path = os.path.join(self.log_dir, f"worker-{actor_id[:8]}.log")
        proc = None
        recycled = self._take_parked(rec.reuse, node, gpu_ids) if rec.reuse and self._poolable(msg) else None
        if recycled is not None:
            proc, conn = recycled
            try:  # the whole environment is replaced (a recycled process carries its last actor's)
                conn.send({"op": "assign", "env": env, "replace": True, "cwd": msg.get("cwd") or os.getcwd(),
                           "log": log_path})
                conn.close()
            except (OSError, EOFError):
                proc = None
        pooled = self._take_pooled() if self._poolable(msg) and proc is None else None
        if pooled is not None:
            proc, conn = pooled
            # the actor-specific part of the environment (a pooled process already
            # carries the head's); applied before the worker touches any GPU
            delta = {k: v for k, v in env.items() if os.environ.get(k) != v}
            unset = [k for k in os.environ if k not in env]
            try:
                conn.send({"op": "assign", "env": delta, "unset": unset, "cwd": msg.get("cwd") or os.getcwd(),
                           "log": log_path})
                conn.close()
            except (OSError, EOFError):
                proc = None
            threading.Thread(target=self.refill_pool, daemon=True).start()
        if proc is None:
            log = open(log_path, "ab")
            cmd = [sys.executable, "-m", "ray_lightning_accelerators_amd.runtime.worker"]
            proc = subprocess.Popen(cmd, env=env, stdout=log if msg.get("capture_output", True) else None,
                                    stderr=subprocess.STDOUT if msg.get("capture_output", True) else None,
                                    cwd=msg.get("cwd") or os.getcwd(), start_new_session=True)
            log.close()
        rec.proc = proc
        rec.pid = proc.pid
        # wait for the worker to register its listener
        while not rec.registered.wait(timeout=0.2):
            if proc.poll() is not None:
                self._mark_dead(rec, f"worker exited during startup (code {proc.returncode})")
                return {"ok": False, "error": rec.death_cause, "log": self._tail_log(actor_id)}
            if time.time() > deadline:
                self._kill(rec, "startup timeout")
                return {"ok": False, "error": "worker startup timed out"}
        return {"ok": True, "actor_id": actor_id, "address": rec.address, "node_ip": node.ip,
                "gpu_ids": gpu_ids, "pid": rec.pid}

    def _tail_log(self, actor_id: str, n: int = 4000) -> str:
        try:
            with open(os.path.join(self.log_dir, f"worker-{actor_id[:8]}.log"), "rb") as f:
                return f.read()[-n:].decode(errors="replace")
        except OSError:
            return ""

    def _mark_dead(self, rec: ActorRecord, cause: str) -> None:
        with self.lock:
            if rec.state == "DEAD":
                return
            rec.state = "DEAD"
            rec.death_cause = cause
            rec.node.give(rec.req, rec.gpu_ids)
            self.lock.notify_all()
            orphans = [a for a in self.actors.values() if a.owner == rec.actor_id and a.state != "DEAD"]
        # actors created BY a dead actor (e.g. a Tune trial's training workers) die with it
        for o in orphans:
            threading.Thread(target=self._kill, args=(o, f"owner {rec.actor_id[:8]} died"), daemon=True).start()

    # -------------------------------------------------------- recycling
    def _take_parked(self, key: str, node: Node, gpu_ids: List[str]):
        """A parked worker of this key / node / GPU set.  When none is parked yet but
        one is on its way (acknowledged a park moments ago: a sequential sweep's next
        trial asks right after the previous one released it), wait for it briefly
        instead of starting another process (``RLA_PARK_WAIT`` seconds, default 1)."""
        want = sorted(gpu_ids)
        deadline = time.time() + float(os.environ.get("RLA_PARK_WAIT", "1.0"))
        with self.pool_cond:
            while True:
                for i, (proc, conn, k, nd, ids) in enumerate(self.parked):
                    if k == key and nd is node and sorted(ids) == want and proc.poll() is None:
                        del self.parked[i]
                        return proc, conn
                coming = any(k == key and nd is node and sorted(ids) == want and p.poll() is None
                             and pid not in self.prewarming
                             for pid, (p, k, nd, ids) in self.parking.items())
                left = deadline - time.time()
                if not coming or left <= 0 or self.stopping:
                    return None
                self.pool_cond.wait(min(left, 0.05))

    def _park(self, rec: ActorRecord) -> bool:
        """Ask a recyclable actor's worker to reset and wait for a new assignment
        (instead of ending it).  True when the worker acknowledged; the caller then
        marks the actor DEAD (its resources return to the ledger)."""
        proc = rec.proc
        if self.stopping or rec.address is None or proc is None or proc.poll() is not None:
            return False
        with self.pool_lock:
            self.parking[proc.pid] = (proc, rec.reuse, rec.node, list(rec.gpu_ids))
        try:
            c = P.connect(rec.address, self.authkey)
            try:
                c.send({"kind": "park", "call_id": "park", "payload": P.dumps(((), {}))})
                # a worker still busy in a call (failure teardown) is ended instead
                ok = c.conn.poll(float(os.environ.get("RLA_PARK_TIMEOUT", "10"))) and bool(c.recv().get("ok"))
            finally:
                c.close()
        except Exception:  # noqa: BLE001 - any failure: end the process instead
            ok = False
        if not ok:
            with self.pool_lock:
                self.parking.pop(proc.pid, None)
        return ok

    def prewarm(self, key: str) -> dict:
        """Start one recyclable worker per free GPU token that initialises HIP and
        loads the native kernels, then parks under ``key`` (idempotent per token)."""
        started = 0
        for node in self.nodes:
            with self.lock:
                tokens = list(node.free_gpus)
            for tok in tokens:
                tag = (key, node.ip, tok)
                if tag in self.prewarmed or self.stopping:
                    continue
                self.prewarmed.add(tag)
                env = self._pool_env()
                env.update({"HIP_VISIBLE_DEVICES": tok, "CUDA_VISIBLE_DEVICES": tok, "RLA_GPU_IDS": tok,
                            P.ENV_NODE_IP: node.ip, P.ENV_NODE_ADDR: node.address})
                log = open(os.path.join(self.log_dir, "prewarm.log"), "ab")
                proc = subprocess.Popen([sys.executable, "-m", "ray_lightning_accelerators_amd.runtime.worker",
                                         "--prewarm", key], env=env, stdout=log, stderr=subprocess.STDOUT,
                                        start_new_session=True)
                log.close()
                with self.pool_lock:
                    self.parking[proc.pid] = (proc, key, node, [tok])
                    self.prewarming.add(proc.pid)  # seconds away: never waited for
                started += 1
        return {"ok": True, "started": started}

    def _kill(self, rec: ActorRecord, cause: str) -> None:
        if rec.reuse and rec.state == "ALIVE" and self._park(rec):
            self._mark_dead(rec, cause + " (worker recycled)")
            return
        proc = rec.proc
        if proc is not None and proc.poll() is None:
            try:
                os.killpg(proc.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
            try:
                proc.wait(timeout=5)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(proc.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                proc.wait(timeout=5)
        self._mark_dead(rec, cause)

    # ----------------------------------------------------------- handlers
    def handle(self, conn: P.SafeConn) -> None:
        while True:
            try:
                msg = conn.recv()
            except (EOFError, OSError):
                return
            op = msg.get("op")
            try:
                if op == "create_actor":
                    reply = self.create_actor(msg)
                elif op == "pool_ready":
                    # a pre-started worker: keep its connection for the assignment
                    with self.pool_lock:
                        proc = self.pool_starting.pop(int(msg["pid"]), None)
                        if proc is not None and not self.stopping:
                            self.pool_ready.append((proc, conn))
                            return
                    conn.close()
                    return
                elif op == "parked":
                    # a recycled / pre-warmed worker, reset and ready for a new actor
                    with self.pool_lock:
                        ent = self.parking.pop(int(msg["pid"]), None)
                        if ent is not None and not self.stopping and msg.get("ok", True):
                            proc, key, node, ids = ent
                            rec = (proc, conn, key, node, ids)
                            # workers that hold a HIP context are handed out first
                            if msg.get("gpu_ready"):
                                self.parked.insert(0, rec)
                            else:
                                self.parked.append(rec)
                            self.prewarming.discard(proc.pid)
                            self.pool_cond.notify_all()
                            return
                    conn.close()
                    return
                elif op == "prewarm":
                    reply = self.prewarm(str(msg["key"]))
                elif op == "register":
                    rec = self.actors.get(msg["actor_id"])
                    if rec is not None:
                        rec.address = msg["address"]
                        rec.state = "ALIVE"
                        rec.registered.set()
                    reply = {"ok": True}
                elif op == "kill":
                    rec = self.actors.get(msg["actor_id"])
                    if rec is not None:
                        self._kill(rec, msg.get("cause", "killed"))
                    reply = {"ok": True}
                elif op == "actors":
                    with self.lock:
                        reply = {"ok": True, "actors": {
                            a.actor_id: {"ActorID": a.actor_id, "State": a.state, "Name": a.name,
                                         "Pid": a.pid, "NodeIP": a.node.ip, "GPUIds": a.gpu_ids,
                                         "ClassName": a.class_name, "DeathCause": a.death_cause,
                                         "Address": a.address}
                            for a in self.actors.values()}}
                elif op == "resources":
                    with self.lock:
                        tot, av = {}, {}
                        for n in self.nodes:
                            for k, v in n.total.items():
                                tot[k] = tot.get(k, 0.0) + v
                            for k, v in n.avail.items():
                                av[k] = av.get(k, 0.0) + v
                        reply = {"ok": True, "total": tot, "available": av,
                                 "nodes": [{"ip": n.ip, "total": dict(n.total), "available": dict(n.avail)}
                                           for n in self.nodes]}
                elif op == "ping":
                    reply = {"ok": True, "pid": os.getpid()}
                elif op == "shutdown":
                    conn.send({"ok": True})
                    self.shutdown()
                    return
                else:
                    reply = {"ok": False, "error": f"unknown op {op}"}
            except Exception as e:  # noqa: BLE001
                reply = {"ok": False, "error": repr(e)}
            try:
                conn.send(reply)
            except (OSError, EOFError):
                return

    def monitor(self) -> None:
        while not self.stopping:
            time.sleep(0.2)
            with self.lock:
                recs = list(self.actors.values())
            for rec in recs:
                if rec.state != "DEAD" and rec.proc is not None and rec.proc.poll() is not None:
                    self._mark_dead(rec, f"worker process exited with code {rec.proc.returncode}")

    def shutdown(self) -> None:
        self.stopping = True
        for rec in list(self.actors.values()):
            if rec.state != "DEAD":
                self._kill(rec, "runtime shutdown")
        with self.pool_lock:
            idle = [p for p, _ in self.pool_ready] + list(self.pool_starting.values())
            idle += [e[0] for e in self.parked] + [e[0] for e in self.parking.values()]
            self.pool_ready, self.pool_starting, self.parked, self.parking = [], {}, [], {}
        for proc in idle:
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
        try:
            self.listener.close()
        except OSError:
            pass
        os._exit(0)

    def serve(self, ready_fd: Optional[int]) -> None:
        threading.Thread(target=self.monitor, daemon=True).start()
        threading.Thread(target=self.refill_pool, daemon=True).start()
        if ready_fd is not None:
            os.write(ready_fd, (self.address + "\n").encode())
            os.close(ready_fd)
        while not self.stopping:
            try:
                c = self.listener.accept()
            except (OSError, EOFError):
                if self.stopping:
                    break
                continue
            threading.Thread(target=self.handle, args=(P.SafeConn(c),), daemon=True).start()


def parse_nodes(spec: str) -> List[Node]:
    """spec: JSON list of {ip, num_cpus, num_gpus, gpu_ids, resources[, address]}."""
    import json

    nodes = []
    for i, d in enumerate(json.loads(spec)):
        nodes.append(Node(d["ip"], d.get("num_cpus", 1), int(d.get("num_gpus", 0)),
                          [str(x) for x in d.get("gpu_ids", [])], d.get("resources", {}),
                          d.get("address") or P.reachable_address(d["ip"], i)))
    return nodes


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--session-dir", required=True)
    ap.add_argument("--nodes", required=True)
    ap.add_argument("--ready-fd", type=int, default=None)
    ap.add_argument("--parent-pid", type=int, default=None)
    args = ap.parse_args(argv)
    authkey = bytes.fromhex(os.environ[P.ENV_AUTH])
    log_dir = os.path.join(args.session_dir, "logs")
    os.makedirs(log_dir, exist_ok=True)
    head = Head(args.session_dir, authkey, parse_nodes(args.nodes), os.environ.get(P.ENV_SYS_PATH, ""), log_dir)
    if args.parent_pid:
        def watch_parent():
            while True:
                time.sleep(1.0)
                try:
                    os.kill(args.parent_pid, 0)
                except ProcessLookupError:
                    head.shutdown()
        threading.Thread(target=watch_parent, daemon=True).start()
    signal.signal(signal.SIGTERM, lambda *a: head.shutdown())
    head.serve(args.ready_fd)


if __name__ == "__main__":
    main()
