"""Per-rank native communicator (C++ ``_comm`` extension) on top of torch.distributed.

``torch.distributed`` (gloo or RCCL process group) is only the bootstrap and
the CPU data plane here.  On MI355X the data plane is the C++ engine
(csrc/comm/): an RCCL communicator created from a unique id that rank 0
broadcasts over the existing group, plus the xGMI one-shot allreduce over
IPC-mapped peer memory for buckets up to ``xgmi_bytes`` (the MNIST gradient is
one 110-530 KiB bucket -- RCCL's ring protocol latency, not link bandwidth,
dominates there).  Reference behaviour being replaced: c10d ProcessGroupNCCL
(``ray_ddp.py:227-237`` init_ddp_connection) and the DDP/Horovod allreduce
(SURVEY.md §2.7 X3/X11).

Safety rules (a wrong collective can hang 8 GPUs):
* the xGMI path is enabled only if EVERY rank set it up and a validation
  allreduce produced the exact expected sum on every rank (agreed with a
  MIN-allreduce over the bootstrap group) -- otherwise all ranks use RCCL;
* the device-side flag polls are bounded: a dead peer sets an error word
  instead of hanging the GPU; ``check()`` raises it, a watchdog thread aborts
  RCCL on async errors.
"""
from __future__ import annotations

import importlib
import logging
import os
from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..config import get_config

_mod = None
_mod_err: Optional[BaseException] = None
# poll bound of the start-up validation collectives (~seconds with s_sleep polling)
VALIDATION_SPIN = 1 << 22


def native_comm_module():
    global _mod, _mod_err
    if _mod is None and _mod_err is None:
        try:
            _mod = importlib.import_module("ray_lightning_accelerators_amd._comm")
        except BaseException as e:  # noqa: BLE001
            _mod_err = e
    return _mod


def _agree(flag: bool, group=None) -> bool:
    """True only if every rank passes True (MIN over the bootstrap group)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return bool(flag)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class NativeCommunicator:
    """RCCL + xGMI communicator of this rank.  ``allreduce_(t)`` sums in place on
    the current stream (graph-capturable); ``average=True`` divides by world."""

    _serials = 0

    def __init__(self, group=None, device: Optional[int] = None, use_rccl: bool = True,
                 use_xgmi: bool = True, xgmi_bytes: Optional[int] = None, validate: bool = True,
                 spin_limit: Optional[int] = None, watchdog_ms: Optional[int] = None,
                 twoshot_bytes: Optional[int] = None):
        """Unset knobs come from :func:`~ray_lightning_accelerators_amd.config.get_config`
        (``allreduce_algo="rccl"`` disables the xGMI path, ``"oneshot"`` forbids RCCL for
        buckets that fit the one-shot area)."""
        NativeCommunicator._serials += 1
        self.serial = NativeCommunicator._serials  # unique per process (worker reuse audit)
        cfg = get_config()
        self.algo = cfg.allreduce_algo
        xgmi_bytes = cfg.xgmi_bytes if xgmi_bytes is None else xgmi_bytes
        spin_limit = cfg.spin_limit if spin_limit is None else spin_limit
        watchdog_ms = cfg.watchdog_ms if watchdog_ms is None else watchdog_ms
        use_xgmi = use_xgmi and self.algo != "rccl"
        mod = native_comm_module()
        if mod is None:
            raise RuntimeError(f"native comm extension (_comm) unavailable: {_mod_err!r}")
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.device = torch.cuda.current_device() if device is None else int(device)
        self._c = mod.Communicator(self.rank, self.world, self.device)
        self._stream = None
        self.fallbacks: list = []  # paths that failed validation (see _drop_failed_path)
        self.rccl = False
        self.xgmi = False
        if use_rccl and os.environ.get("RLA_DISABLE_RCCL", "0") != "1":
            uid = [mod.Communicator.unique_id() if self.rank == 0 else None]
            if self.world > 1:
                dist.broadcast_object_list(uid, src=0, group=group)
            ok = True
            try:
                self._c.init_rccl(uid[0])
            except RuntimeError:
                ok = False
            self.rccl = _agree(ok, group)
        self.twoshot = False
        if use_xgmi and 1 < self.world <= mod.XGMI_MAX_RANKS and os.environ.get("RLA_DISABLE_XGMI", "0") != "1":
            self._setup_xgmi(xgmi_bytes, validate, spin_limit, group)
            tbytes = cfg.twoshot_bytes if twoshot_bytes is None else twoshot_bytes
            if tbytes > 0 and self.algo in ("auto", "twoshot"):
                self._setup_twoshot(tbytes, validate, spin_limit, group)
        # routing limits of the C++ side (reducer / fusion engine / allreduce_f32):
        # "oneshot" never uses two-shot, "twoshot" never uses one-shot
        one_max = 0 if self.algo == "twoshot" else (1 << 62)
        two_max = 0 if self.algo == "oneshot" else (1 << 62)
        self._c.set_route_limits(one_max, two_max)
        if watchdog_ms > 0:
            self._c.start_watchdog(watchdog_ms)
        if self.rank == 0:
            # the data-plane decision of this job, once
            logging.getLogger("ray_lightning_accelerators_amd.comm").info("bring-up: %s", self.describe())

    # ------------------------------------------------------------- xGMI
    def _setup_xgmi(self, xgmi_bytes, validate, spin_limit, group):
        ok = True
        handle = b""
        try:
            handle = self._c.xgmi_handle(max(4, xgmi_bytes // 4))
        except RuntimeError:
            ok = False
        handles = [None] * self.world
        dist.all_gather_object(handles, handle if ok else b"", group=group)
        ok = ok and all(h for h in handles)
        if ok:
            try:
                self._c.xgmi_open(handles)
            except RuntimeError:
                ok = False
        if not _agree(ok, group):
            return
        if validate:
            # short bounded polls while validating: every rank launches right after a
            # barrier, so a broken link shows up in seconds, not after the (minutes-
            # long) training bound
            self._c.set_spin_limit(min(int(spin_limit or VALIDATION_SPIN), VALIDATION_SPIN))
            ok = self._validate_xgmi(group)
            if not _agree(ok, group):
                self._drop_failed_path(0, "xGMI one-shot", group)
                return
        if spin_limit is not None:
            self._c.set_spin_limit(int(spin_limit))
        self.xgmi = True

    def _drop_failed_path(self, which: int, name: str, group) -> None:
        """A validation failed on some rank: take the path out of the C++ router on
        EVERY rank and clear a latched poll timeout, so the fallback (two-shot /
        RCCL / c10d) starts from a healthy communicator.  Collective."""
        torch.cuda.synchronize(self.device)  # a timed-out kernel has drained by now
        dist.barrier(group=group)
        self._c.disable_path(which)
        self._c.reset_error()
        dist.barrier(group=group)
        self.fallbacks.append(name)
        if self.rank == 0:
            import sys

            print(f"[rla.comm] {name} failed validation on some rank; falling back", file=sys.stderr, flush=True)

    def _fault_validation(self) -> bool:
        """Fault injection (tests): ``RLA_FAULT_XGMI_VALIDATION=<rank>`` makes that
        rank skip its validation launches, so its peers' polls time out exactly as
        they would over a broken link."""
        return os.environ.get("RLA_FAULT_XGMI_VALIDATION", "") == str(self.rank)

    def _validate_xgmi(self, group) -> bool:
        n = min(4096 + 4, int(self._c.xgmi_capacity))
        dev = torch.device("cuda", self.device)
        ok = True
        for it in range(3):  # both receive-area parities + one reuse
            x = (torch.arange(n, device=dev, dtype=torch.float32) % 97) * (self.rank + 1) + it
            want = (torch.arange(n, device=dev, dtype=torch.float32) % 97) * (self.world * (self.world + 1) / 2) \
                + it * self.world
            torch.cuda.synchronize(dev)
            dist.barrier(group=group)
            if self._fault_validation():
                ok = False  # the peers' kernels time out waiting for this rank's push
                continue
            try:
                self._c.allreduce_xgmi(x)
                torch.cuda.synchronize(dev)
            except RuntimeError:
                return False
            ok = ok and self._c.error_state() == 0 and bool(torch.equal(x, want))
        return ok

    def _setup_twoshot(self, tbytes, validate, spin_limit, group):
        """Two-shot region (reduce-scatter + all-gather over xGMI) for buckets above
        the one-shot area; same all-or-nothing agreement as the one-shot."""
        ok = True
        handle = b""
        try:
            handle = self._c.twoshot_handle(max(4 * self.world, int(tbytes) // 4))
        except RuntimeError:
            ok = False
        handles = [None] * self.world
        dist.all_gather_object(handles, handle if ok else b"", group=group)
        ok = ok and all(h for h in handles)
        if ok:
            try:
                self._c.twoshot_open(handles)
            except RuntimeError:
                ok = False
        if not _agree(ok, group):
            return
        if validate:
            self._c.set_spin_limit(min(int(spin_limit or VALIDATION_SPIN), VALIDATION_SPIN))
            ok = self._validate_twoshot(group)
            if not _agree(ok, group):
                self._drop_failed_path(1, "xGMI two-shot", group)
                return
        if spin_limit is not None:
            self._c.set_spin_limit(int(spin_limit))
        self.twoshot = True

    def _validate_twoshot(self, group) -> bool:
        dev = torch.device("cuda", self.device)
        ok = True
        # both parities, a reuse, a ragged size (chunk tails) and a bf16-wire pass
        big = min(8192 * self.world + 12, int(self._c.twoshot_capacity))
        for it, n in enumerate((big, min(4097, big), big)):
            base = torch.arange(n, device=dev, dtype=torch.float32) % 97
            x = base * (self.rank + 1) + it
            want = base * (self.world * (self.world + 1) / 2) + it * self.world
            torch.cuda.synchronize(dev)
            dist.barrier(group=group)
            if self._fault_validation():
                ok = False
                continue
            try:
                self._c.allreduce_twoshot(x, False)
                torch.cuda.synchronize(dev)
            except RuntimeError:
                return False
            ok = ok and self._c.error_state() == 0 and bool(torch.equal(x, want))
        x = torch.full((min(4100, big),), float(self.rank + 1), device=dev)
        dist.barrier(group=group)
        if self._fault_validation():
            return False
        try:
            self._c.allreduce_twoshot(x, True)  # small integers are exact in bf16
            torch.cuda.synchronize(dev)
        except RuntimeError:
            return False
        return ok and self._c.error_state() == 0 and bool(torch.all(x == self.world * (self.world + 1) / 2))

    @property
    def xgmi_capacity(self) -> int:
        return int(self._c.xgmi_capacity) if self.xgmi else 0

    @property
    def twoshot_capacity(self) -> int:
        return int(self._c.twoshot_capacity) if self.twoshot else 0

    def route(self, t: torch.Tensor) -> str:
        """Which path ``allreduce_`` takes for this fp32 GPU tensor."""
        if self.world == 1:
            return "none"
        if self.xgmi or self.twoshot:
            r = int(self._c.route(t))
            if r >= 0 and not (r == 2 and not self.rccl):
                return ("oneshot", "twoshot", "rccl", "twoshot")[r]  # 3: region-sized pieces
        return "rccl" if self.rccl else "torch"

    def dp_context(self, capacity_floats: int) -> Optional[list]:
        """Open the auxiliary peer region that a compute kernel exchanges through
        directly (the fused data-parallel MLP tail pushes its gradient tiles into
        every peer's receive area from its Adam epilogue).  Collective; returns the
        kernel context ``[world, rank, stride, spin, gen, err, region_0..]`` or None
        on every rank when any rank could not map the peers (caller falls back to
        the communicator's allreduce)."""
        if not self.xgmi or self.world == 1:
            return None
        if self._c.has_aux:
            return list(self._c.aux_context())
        ok = True
        handle = b""
        try:
            handle = self._c.aux_handle(int(capacity_floats))
        except RuntimeError:
            ok = False
        handles = [None] * self.world
        dist.all_gather_object(handles, handle if ok else b"", group=self.group)
        ok = ok and all(h for h in handles)
        if ok:
            try:
                self._c.aux_open(handles)
            except RuntimeError:
                ok = False
        if not _agree(ok, self.group):
            return None
        return list(self._c.aux_context())

    def dp_rearm(self) -> None:
        """Re-arm the auxiliary region for a new exchange protocol (collective): every
        rank drains its device, no kernel of any peer can still be writing, each rank
        resets its own region (tags that match no coming step, generations 0)."""
        if not self._c.has_aux:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        self._c.aux_rearm()
        dist.barrier(group=self.group)
        self.rearms = getattr(self, "rearms", 0) + 1

    # ------------------------------------------------------- collectives
    def allreduce_(self, t: torch.Tensor, average: bool = False, bf16_wire: bool = False) -> torch.Tensor:
        """In-place SUM (``average``: mean).  fp32 GPU buckets go through the C++
        router: xGMI one-shot (small), xGMI two-shot (medium/large), RCCL (rest).
        ``bf16_wire``: carry bf16 over the links (two-shot; fp32 accumulate)."""
        if self.world == 1:
            return t
        fp32 = t.dtype == torch.float32 and t.is_cuda and t.is_contiguous()
        if bf16_wire and fp32 and self.twoshot and self._c.allreduce_bf16wire(t):
            pass
        elif bf16_wire and fp32:
            w = t.to(torch.bfloat16)  # no two-shot region for it: compress around the generic path
            self.allreduce_(w)
            t.copy_(w)
        elif fp32 and (self.xgmi or self.twoshot) and self.route(t) in ("oneshot", "twoshot", "rccl"):
            self._c.allreduce_f32(t)
        elif self.rccl:
            self._c.allreduce(t, 0)
        elif t.is_cuda and dist.get_backend(self.group) == "gloo":
            tmp = t.cpu()  # CPU bootstrap group: not graph-capturable, correctness path only
            dist.all_reduce(tmp, group=self.group)
            t.copy_(tmp)
        else:
            dist.all_reduce(t, group=self.group)
        if average:
            t.div_(self.world)
        return t

    def allreduce_async(self, t: torch.Tensor, average: bool = False,
                        probe: Optional[torch.Tensor] = None, bf16_wire: bool = False) -> "_StreamWork":
        """Allreduce on this communicator's high-priority side stream, ordered after
        the current stream's pending work (the gradient producer); ``wait()``
        makes the then-current stream wait for it -- DDP bucket overlap.
        ``probe`` (fp64 [4], debug): slots 1 / 2 receive the checksum of ``t`` as
        the comm stream sees it before / after the collective."""
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=t.device, priority=-1)
        cur = torch.cuda.current_stream(t.device)
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            if probe is not None:
                probe[1] = t.double().sum()
            self.allreduce_(t, average=average, bf16_wire=bf16_wire)
            if probe is not None:
                probe[2] = t.double().sum()
                probe.record_stream(self._stream)
        ev = torch.cuda.Event()
        ev.record(self._stream)
        t.record_stream(self._stream)
        return _StreamWork(ev)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world == 1:
            return t
        if self.rccl:
            self._c.broadcast(t, src)
        else:
            dist.broadcast(t, src, group=self.group)
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        if self.rccl:
            self._c.allgather(t.contiguous(), out)
        else:
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out.view(self.world, *t.shape)

    def reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        assert t.numel() % self.world == 0
        out = torch.empty(t.numel() // self.world, dtype=t.dtype, device=t.device)
        if self.rccl:
            self._c.reduce_scatter(t.contiguous(), out, 0)
        else:
            dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
        return out

    def fusion_engine(self, fusion_bytes: int = 8 << 20):
        return native_comm_module().FusionEngine(self._c, int(fusion_bytes), self.device)

    # ------------------------------------------------------------ health
    def check(self) -> None:
        st = self._c.error_state()
        if st != 0:
            raise RuntimeError(f"collective failure on rank {self.rank}: {self._c.error_message()}")

    def abort(self) -> None:
        self._c.abort()

    def describe(self) -> str:
        return (f"NativeCommunicator(rank={self.rank}, world={self.world}, rccl={self.rccl}, "
                f"xgmi={self.xgmi}, xgmi_capacity={self.xgmi_capacity}, twoshot={self.twoshot}, "
                f"twoshot_capacity={self.twoshot_capacity}, failed_validation={self.fallbacks})")


class _StreamWork:
    """c10d-Work-like handle of a side-stream collective."""

    def __init__(self, event: "torch.cuda.Event"):
        self.event = event

    def wait(self) -> bool:
        torch.cuda.current_stream().wait_event(self.event)
        return True

    def is_completed(self) -> bool:
        return self.event.query()


_default: Optional[NativeCommunicator] = None


def get_native_comm(create: bool = True, **kw) -> Optional[NativeCommunicator]:
    """Process-wide communicator for the default group (GPU ranks only)."""
    global _default
    if _default is None and create and torch.cuda.is_available() and dist.is_initialized() \
            and get_config().native_comm and get_config().allreduce_algo != "torch" \
            and native_comm_module() is not None:
        _default = NativeCommunicator(**kw)
    return _default


def reset_native_comm() -> None:
    global _default
    if _default is not None:
        try:
            torch.cuda.synchronize(_default.device)
        except Exception:  # noqa: BLE001 - teardown must not raise
            pass
    _default = None  # the C++ destructor destroys the RCCL comm and unmaps peers


def allreduce_async(t: torch.Tensor, group=None):
    """Async SUM allreduce: native side-stream collective for GPU tensors on the
    default group when the native engine is up, else c10d's async work."""
    if group is None and t.is_cuda:
        comm = get_native_comm()
        if comm is not None:
            return comm.allreduce_async(t)
    return dist.all_reduce(t, group=group, async_op=True)


def make_allreduce(average: bool = False, prefer_native: bool = True) -> Callable[[torch.Tensor], torch.Tensor]:
    """Best available in-place SUM (or mean) allreduce for this process."""
    comm = get_native_comm() if prefer_native else None
    if comm is not None:
        return lambda t: comm.allreduce_(t, average=average)

    def _f(t):
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(t)
            if average:
                t.div_(dist.get_world_size())
        return t
    return _f
