"""Small utilities of the Lightning-compatible layer: seeding, atomic save,
rank-zero helpers, logging.  (Reference call sites: PL_GLOBAL_SEED propagation
ray_ddp.py:154-159; atomic_save tune.py:5,133 of the reference.)"""
from __future__ import annotations

import logging
import os
import random
import sys
import time
import tempfile
from functools import wraps
from typing import Any, Optional

import numpy as np
import torch

log = logging.getLogger("ray_lightning_accelerators_amd")
if not log.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("%(levelname)s %(name)s: %(message)s"))
    log.addHandler(_h)
    log.setLevel(logging.WARNING)


def seed_everything(seed: Optional[int] = None, workers: bool = False) -> int:
    """Seed python, numpy and torch; exported as ``PL_GLOBAL_SEED`` so the
    accelerators can forward it to their workers (reference ray_ddp.py:154-159)."""
    if seed is None:
        env = os.environ.get("PL_GLOBAL_SEED")
        seed = int(env) if env is not None else random.randint(0, 2 ** 31 - 1)
    seed = int(seed)
    os.environ["PL_GLOBAL_SEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    if workers:
        os.environ["PL_SEED_WORKERS"] = "1"
    return seed


def reset_seed() -> None:
    seed = os.environ.get("PL_GLOBAL_SEED")
    if seed is not None:
        seed_everything(int(seed))


def atomic_save(checkpoint: Any, filepath: str) -> None:
    """torch.save to a temp file in the same directory, then rename (atomic on POSIX)."""
    d = os.path.dirname(os.path.abspath(filepath)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp_ckpt_", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(checkpoint, f)
        os.replace(tmp, filepath)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def _private_copy(obj: Any) -> Any:
    """The checkpoint dict with every tensor cloned, so a background write never
    reads storage the training loop keeps mutating (``.cpu()`` of a CPU tensor is
    the tensor itself)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().clone()
    if isinstance(obj, dict):  # dict / OrderedDict (state dicts)
        return type(obj)((k, _private_copy(v)) for k, v in obj.items())
    if type(obj) in (list, tuple):
        return type(obj)(_private_copy(v) for v in obj)
    return obj


class CheckpointWriter:
    """One background thread that runs checkpoint file operations in submission
    order (writes and the top-k removals that must follow them), so the epoch-end
    checkpoint write (~1.7 ms for the MNIST model: pickling + file I/O) overlaps
    the next epoch's GPU work instead of stalling it.  ``wait()`` drains the
    queue and re-raises the first error; the Trainer waits before ``fit``
    returns and before any synchronous save."""

    def __init__(self):
        import queue
        import threading

        self._q: "queue.Queue" = queue.Queue()
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._loop, name="rla-ckpt-writer", daemon=True)
        self._t.start()

    def _loop(self) -> None:
        while True:
            item = self._q.get()
            try:
                if item is None:
                    return
                fn, args = item
                if self._err is None:
                    fn(*args)
            except BaseException as e:  # noqa: BLE001 - surfaced by wait()
                self._err = e
            finally:
                self._q.task_done()

    def submit(self, fn, *args) -> None:
        self._raise()
        self._q.put((fn, args))

    def save(self, checkpoint: Any, filepath: str) -> None:
        self.submit(atomic_save, _private_copy(checkpoint), filepath)

    def wait(self) -> None:
        self._q.join()
        self._raise()

    def _raise(self) -> None:
        if self._err is not None:
            e, self._err = self._err, None
            raise RuntimeError(f"background checkpoint write failed: {e!r}") from e

    def close(self) -> None:
        self.wait()
        self._q.put(None)
        self._t.join(timeout=10)


def _flatten_tensors(obj: Any, out: list) -> Any:
    """Replace every tensor of a (nested) checkpoint dict by a placeholder; collect them."""
    if isinstance(obj, torch.Tensor):
        out.append(obj)
        return _TensorSlot(len(out) - 1)
    if isinstance(obj, dict):
        return type(obj)((k, _flatten_tensors(v, out)) for k, v in obj.items())
    if type(obj) in (list, tuple):
        return type(obj)(_flatten_tensors(v, out) for v in obj)
    return obj


class _TensorSlot:
    __slots__ = ("i",)

    def __init__(self, i: int):
        self.i = i


def _rebuild_tensors(obj: Any, tensors: list) -> Any:
    if isinstance(obj, _TensorSlot):
        return tensors[obj.i]
    if isinstance(obj, dict):
        return type(obj)((k, _rebuild_tensors(v, tensors)) for k, v in obj.items())
    if type(obj) in (list, tuple):
        return type(obj)(_rebuild_tensors(v, tensors) for v in obj)
    return obj


def _writer_main(conn) -> None:  # pragma: no cover - runs in the writer process
    """Checkpoint writer process: rebuild each checkpoint from the shared-memory
    block it names, ``atomic_save`` it, run file removals, in submission order."""
    import pickle
    from multiprocessing import shared_memory

    import threading

    # a forked writer must not enter a parallel region: the parent's OpenMP pool
    # threads do not exist in the child (an intra-op parallel copy would wait on them)
    torch.set_num_threads(1)
    lock = threading.Lock()
    busy = threading.Event()

    def send(m):
        with lock:
            conn.send(m)

    def beat():
        # while a request is in progress, a "beat" every BEAT_S: a large checkpoint on
        # a slow filesystem is busy, not stalled (the trainer's stall timer
        # restarts at every message)
        while True:
            busy.wait()
            time.sleep(ProcessCheckpointWriter.BEAT_S)
            if busy.is_set():
                try:
                    send(("beat", None))
                except (OSError, EOFError, BrokenPipeError):
                    return

    threading.Thread(target=beat, daemon=True, name="rla-ckpt-writer-beat").start()
    send(("ready", None))
    while True:
        try:
            msg = conn.recv()
        except EOFError:
            return
        op = msg[0]
        err = None
        busy.set()
        try:
            if op == "save":
                _, skel, metas, shm_name, filepath = msg
                shm = shared_memory.SharedMemory(name=shm_name)
                try:  # attaching registered it with the tracker (py3.10); the trainer owns it
                    from multiprocessing import resource_tracker

                    resource_tracker.unregister(shm._name, "shared_memory")
                except Exception:  # noqa: BLE001
                    pass
                try:
                    buf = torch.frombuffer(shm.buf, dtype=torch.uint8)
                    tensors = [buf[off: off + nb].view(dt).reshape(shape).clone() for dt, shape, off, nb in metas]
                    del buf
                finally:
                    shm.close()
                atomic_save(_rebuild_tensors(pickle.loads(skel), tensors), filepath)
            elif op == "remove":
                if os.path.exists(msg[1]):
                    try:
                        os.remove(msg[1])
                    except OSError:
                        pass
            elif op == "sleep":  # test hook: a long request (heartbeat test)
                time.sleep(float(msg[1]))
            elif op == "exit":
                busy.clear()
                send(("done", None))
                return
        except BaseException as e:  # noqa: BLE001 - reported to the trainer
            err = repr(e)
        busy.clear()
        send(("done", err))


class ProcessCheckpointWriter:
    """Checkpoint files written by a separate process, in submission order.

    The training process only copies the checkpoint's (host) tensors into one
    shared-memory block and sends a small pickled skeleton; pickling the tensors,
    the file write and the atomic rename happen in the writer process -- on
    another core, off the GIL -- while the training process dispatches the next
    epoch.  (A writer THREAD competed with the dispatching thread for the GIL and
    made the MNIST epoch 0.7 ms longer, profiles/r2_c38.)  The writer starts with
    the first save (``spawn``: a fresh interpreter, never a fork of a process that
    holds a GPU context); files are identical to ``atomic_save``'s."""

    def __init__(self, force_spawn: bool = False):
        self._start(force_spawn)
        self._pending = []  # (shared-memory block or None, request) of unacknowledged requests
        self._err: Optional[str] = None

    def _start(self, force_spawn: bool) -> None:
        import multiprocessing as mp

        # fork (instant: torch is already imported) only while this process holds no
        # GPU context; otherwise spawn a fresh interpreter (~1-2 s until ready())
        torch_mod = sys.modules.get("torch")
        gpu_ctx = force_spawn or (torch_mod is not None and torch_mod.cuda.is_initialized())
        if not gpu_ctx:
            from ..utils import warmup

            warmup.join()  # never fork while a warm-up thread may hold an import lock
        if not gpu_ctx:
            # everything the writer imports, imported HERE first: a forked child that
            # imports a module another thread of this process was importing at the
            # fork inherits that module's import lock held -- and waits on it forever
            import pickle  # noqa: F401
            from multiprocessing import resource_tracker, shared_memory  # noqa: F401
        ctx = mp.get_context("spawn" if gpu_ctx else "fork")
        self._conn, child = ctx.Pipe()
        self._proc = ctx.Process(target=_writer_main, args=(child,), daemon=True, name="rla-ckpt-writer")
        self._proc.start()
        child.close()
        self._ready = False
        self._dead = False
        self._started_at = time.monotonic()

    def ready(self) -> bool:
        """The writer finished starting (interpreter + torch import, ~1-2 s)."""
        while not self._ready and self._proc.is_alive() and self._conn.poll():
            try:
                self._ready = self._conn.recv()[0] == "ready"
            except EOFError:
                break
        return self._ready

    def alive(self) -> bool:
        return not self._dead and self._proc.is_alive()

    # a writer silent this long while requests are pending is declared stuck: it is
    # killed and the pending requests are completed in this process (a Tune sweep
    # once hung here for good, profiles/r4_tune/cfg4_recycle_stalled_run.log).  A busy
    # writer sends a "beat" every BEAT_S, so only true silence counts; its start-up
    # (a spawned interpreter importing torch on a loaded box) gets STARTUP_S
    STALL_S = 20.0
    BEAT_S = 1.0
    STARTUP_S = 180.0

    def _recv(self, block: bool):
        """The writer's next message (heartbeats skipped), or None (non-blocking and
        nothing there); raises EOFError when the writer died or stayed silent past
        STALL_S (STARTUP_S before its ready message)."""
        while True:
            if not block:
                if not self._conn.poll():
                    return None
            else:
                limit = self.STALL_S if self._ready else max(
                    self.STALL_S, self.STARTUP_S - (time.monotonic() - self._started_at))
                if not self._conn.poll(limit):
                    raise EOFError("checkpoint writer process stalled")
            msg = self._conn.recv()
            if msg[0] != "beat":
                return msg

    def _reap(self, block: bool) -> None:
        try:
            if self._pending and not self._ready:
                msg = self._recv(block)
                if msg is None:
                    return
                self._ready = msg[0] == "ready"
            while self._pending:
                msg = self._recv(block)
                if msg is None:
                    return
                shm, _req = self._pending.pop(0)
                if shm is not None:
                    shm.close()
                    shm.unlink()
                if msg[1] and self._err is None:
                    self._err = msg[1]
        except EOFError:
            self._take_over()

    def _take_over(self) -> None:
        """The writer died or stalled: stop it and finish its queue here, in order."""
        import pickle

        global writer_takeovers
        writer_takeovers += 1
        print(f"[rla] checkpoint writer process {self._proc.pid} stopped answering; "
              f"finishing {len(self._pending)} request(s) in-process", file=sys.stderr, flush=True)

        try:
            self._proc.terminate()
            self._proc.join(timeout=5)
            if self._proc.is_alive():
                self._proc.kill()
                self._proc.join(timeout=5)
        except Exception:  # noqa: BLE001
            pass
        self._dead = True
        pending, self._pending = self._pending, []
        if self._proc.is_alive():
            # never replay while the old writer may still finish a rename: a replayed
            # removal could race its save and resurrect a deleted top-k file
            for shm, _req in pending:
                if shm is not None:
                    shm.close()
                    shm.unlink()
            if self._err is None:
                self._err = f"checkpoint writer process {self._proc.pid} could not be stopped"
            return
        for shm, req in pending:
            try:
                if req is not None and req[0] == "save":
                    _, skel, metas, _name, filepath = req
                    buf = torch.frombuffer(shm.buf, dtype=torch.uint8)
                    tensors = [buf[o: o + nb].view(dt).reshape(shape).clone() for dt, shape, o, nb in metas]
                    del buf
                    atomic_save(_rebuild_tensors(pickle.loads(skel), tensors), filepath)
                elif req is not None and req[0] == "remove" and os.path.exists(req[1]):
                    os.remove(req[1])
            except BaseException as e:  # noqa: BLE001 - reported like the writer's errors
                if self._err is None:
                    self._err = repr(e)
            finally:
                if shm is not None:
                    shm.close()
                    shm.unlink()
        # a fresh writer for the saves to come (spawned: safe from any thread, and
        # this process may hold a GPU context); until it is ready, saves queue on it
        try:
            self._conn.close()
        except Exception:  # noqa: BLE001
            pass
        try:
            self._start(force_spawn=True)
        except Exception:  # noqa: BLE001 - no writer: later saves run in-process
            self._dead = True

    def save(self, checkpoint: Any, filepath: str) -> None:
        import pickle
        from multiprocessing import shared_memory

        self._reap(block=False)
        self._raise()
        tensors: list = []
        skel = pickle.dumps(_flatten_tensors(checkpoint, tensors), protocol=pickle.HIGHEST_PROTOCOL)
        metas, off = [], 0
        flat = [t.detach().cpu().contiguous() for t in tensors]
        for t in flat:
            nb = t.numel() * t.element_size()
            metas.append((t.dtype, tuple(t.shape), off, nb))
            off += (nb + 63) // 64 * 64
        shm = shared_memory.SharedMemory(create=True, size=max(off, 64))
        try:
            buf = torch.frombuffer(shm.buf, dtype=torch.uint8)
            for t, (_, _, o, nb) in zip(flat, metas):
                if nb:
                    buf[o: o + nb].copy_(t.reshape(-1).view(torch.uint8))
            del buf
        except BaseException:
            shm.close()
            shm.unlink()
            raise
        # absolute: the writer process keeps the directory it started in, while this
        # process changes it (a recycled worker per assignment, a Tune trial per trial)
        req = ("save", skel, metas, shm.name, os.path.abspath(filepath))
        self._pending.append((shm, req))
        if self._dead:
            self._take_over()
            self._raise()
            return
        try:
            self._conn.send(req)
        except (OSError, EOFError, BrokenPipeError):
            self._take_over()

    def submit(self, fn, *args) -> None:
        """File operations after the pending writes (only removals are shipped)."""
        if getattr(fn, "__name__", "") == "_remove_file" and len(args) == 1 and not self._dead:
            req = ("remove", os.path.abspath(args[0]))
            self._pending.append((None, req))
            try:
                self._conn.send(req)
            except (OSError, EOFError, BrokenPipeError):
                self._take_over()
        else:
            self.wait()
            fn(*args)

    def wait(self) -> None:
        self._reap(block=True)
        self._raise()

    def _raise(self) -> None:
        if self._err is not None:
            e, self._err = self._err, None
            raise RuntimeError(f"background checkpoint write failed: {e}")

    def close(self) -> None:
        try:
            self.wait()
        finally:
            if not self._dead:
                try:
                    self._pending.append((None, None))
                    self._conn.send(("exit",))
                    self._reap(block=True)
                except (OSError, EOFError):
                    pass
            self._proc.join(timeout=10)


_process_writer: Optional[ProcessCheckpointWriter] = None
writer_takeovers = 0  # writer processes this process had to take over (diagnostics)


def process_checkpoint_writer() -> ProcessCheckpointWriter:
    """The process-wide checkpoint writer (started on first use; a recycled training
    worker keeps it across fits, so short Tune trials do not each pay its start-up)."""
    global _process_writer
    if _process_writer is None or not _process_writer.alive():
        _process_writer = ProcessCheckpointWriter()
    return _process_writer


def load_checkpoint(path: str, map_location: Any = "cpu") -> dict:
    """Load a Lightning checkpoint.  Files written by this framework contain
    only tensors/containers/primitives, so the safe ``weights_only`` loader is
    tried first; hparams objects of user classes fall back to a full load of
    OUR OWN files only (never used on third-party files)."""
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except Exception:
        return torch.load(path, map_location=map_location, weights_only=False)


class _RankZero:
    rank = 0


rank_zero_only_state = _RankZero()


def rank_zero_only(fn):
    @wraps(fn)
    def wrapped(*args, **kwargs):
        if rank_zero_only_state.rank == 0:
            return fn(*args, **kwargs)
        return None

    wrapped.rank = 0
    return wrapped


@rank_zero_only
def rank_zero_warn(msg: str) -> None:
    log.warning(msg)


@rank_zero_only
def rank_zero_info(msg: str) -> None:
    log.info(msg)


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def move_to_device(batch: Any, device: torch.device, non_blocking: bool = True) -> Any:
    if isinstance(batch, torch.Tensor):
        return batch.to(device, non_blocking=non_blocking)
    if isinstance(batch, (list, tuple)):
        out = [move_to_device(b, device, non_blocking) for b in batch]
        return type(batch)(out) if not hasattr(batch, "_fields") else type(batch)(*out)
    if isinstance(batch, dict):
        return {k: move_to_device(v, device, non_blocking) for k, v in batch.items()}
    return batch


def to_float(v: Any) -> float:
    if isinstance(v, torch.Tensor):
        return float(v.detach().float().mean().item())
    return float(v)
