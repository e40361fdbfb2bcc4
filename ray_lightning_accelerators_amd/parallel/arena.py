"""Flat parameter / gradient arenas (SURVEY.md §7 decision D3).

Every floating-point parameter of a module becomes a view into ONE contiguous
fp32 buffer per device, and its ``.grad`` a view into a parallel gradient
buffer.  Consequences on MI355X:
  * the optimizer step is one fused HIP launch over the arena
    (``ops.fused_adam_`` / ``ops.fused_sgd_``) instead of a multi-tensor apply;
  * DDP buckets are contiguous arena slices, so the allreduce runs in place
    with no flatten/unflatten copies (the reference's DDP reducer copies every
    grad into a bucket and back);
  * checkpoints still see ordinary per-parameter tensors (views).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
from torch import nn


class ParamArena:
    """``steal_grads`` (default on GPU): ``zero_grad`` sets ``.grad = None`` so
    autograd hands over freshly produced gradient tensors (no zero-fill of the
    arena, no per-parameter accumulate kernel -- ResNet-50 has 161 of them), and
    :meth:`gather_grads` moves a whole bucket / step of them into the arena with
    ONE multi-tensor copy launch whose chunk table is cached per address set."""

    def __init__(self, module: nn.Module, params: Optional[List[nn.Parameter]] = None, align: int = 4,
                 steal_grads: Optional[bool] = None):
        if params is None:
            params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        dev = params[0].device
        for p in params:
            if p.device != dev:
                raise ValueError("all parameters of an arena must live on one device")
            if p.dtype != torch.float32:
                raise ValueError(f"arena parameters must be fp32 master weights, got {p.dtype}")
        self.device = dev
        self.params = params
        # offsets aligned to 4 elements (16 B) so every view is float4-aligned
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for p in params:
            n = p.numel()
            self.offsets.append((off, n))
            off += (n + align - 1) // align * align
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        # each view keeps its parameter's memory format: a channels_last conv weight
        # stays channels_last (NHWC convolutions would otherwise re-layout -- clone --
        # every bf16 weight on every use, and its channels_last gradient would need a
        # strided copy into a contiguous arena view; profiles/r3_rn50)
        self.strides: List[Optional[Tuple[int, ...]]] = [
            tuple(p.stride()) if (not p.is_contiguous() and p.dim() == 4
                                  and p.is_contiguous(memory_format=torch.channels_last)) else None
            for p in params]
        with torch.no_grad():
            for i, (p, (o, n)) in enumerate(zip(params, self.offsets)):
                view = self._shaped(self.data, i, p)
                view.copy_(p.data)
                p.data = view
                p.grad = self._shaped(self.grad, i, p)
        self._index: Dict[int, int] = {id(p): i for i, p in enumerate(params)}
        self.bf16: Optional[torch.Tensor] = None  # bf16 weight shadow (enable_bf16_shadow)
        self._shadow_ver = -1
        self._pver = 0
        self.steal_grads = (dev.type == "cuda") if steal_grads is None else bool(steal_grads)
        self._tables: "OrderedDict[tuple, torch.Tensor]" = OrderedDict()
        self._graph_tables: List[tuple] = []
        self._graph_staging: Optional[torch.Tensor] = None
        self._graph_staging_off = 0

    def _shaped(self, flat: torch.Tensor, i: int, like: torch.Tensor, base: int = 0) -> torch.Tensor:
        o, n = self.offsets[i]
        st = self.strides[i]
        seg = flat[o - base:o - base + n]
        if st is None:
            return seg.view_as(like)
        return seg.as_strided(like.shape, st)

    def shaped_slice(self, flat: torch.Tensor, i: int, base: int = 0) -> torch.Tensor:
        """Parameter ``i``'s segment of a buffer laid out like the arena (optimizer
        state; ``flat`` starts at arena element ``base``), in the parameter's layout."""
        return self._shaped(flat, i, self.params[i], base)

    # ------------------------------------------------------ bf16 weight shadow
    def enable_bf16_shadow(self, module: Optional[nn.Module] = None) -> None:
        """Keep a bf16 copy of every parameter, written by the fused optimizer step
        in the same pass as the fp32 update: bf16 compute (autocast) reads it instead
        of casting each weight in every forward (ResNet-50: 56 cast kernels a step).
        ``module``: the root whose forward re-checks the parameters' version counters
        (an outside write -- load_state_dict, a manual edit -- refreshes the shadow)."""
        if self.bf16 is None:
            self.bf16 = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            self.refresh_bf16()
            from ..ops import shadow

            shadow.register(self)
            if module is not None:
                module.register_forward_pre_hook(lambda mod, args: self.check_bf16())

    def invalidate_bf16(self) -> None:
        """The fp32 weights were written behind the version counters (a collective)."""
        self._shadow_ver = -1

    def _param_version(self) -> int:
        # a parameter's own counter (load_state_dict's copy_, in-place edits) plus the
        # arena buffer's (writes through arena slices, e.g. rebind_all)
        return sum(p._version for p in self.params) + self.data._version

    def check_bf16(self) -> None:
        if self.bf16 is not None and self._param_version() != self._shadow_ver:
            self.refresh_bf16()

    def refresh_bf16(self) -> None:
        with torch.no_grad():
            self.bf16.copy_(self.data)
        self._shadow_ver = self._param_version()
        self._pver = self._shadow_ver - self.data._version  # per-parameter part at refresh

    def bf16_weight(self, p: torch.Tensor) -> Optional[torch.Tensor]:
        """``p``'s bf16 shadow (parameter layout), refreshed first when the fp32
        weights changed outside the fused step (load_state_dict, broadcast, manual
        edits -- every such write bumps the parameters' shared version counter; the
        fused step writes through raw pointers and bumps nothing).  None when ``p``
        is not in the arena or there is no shadow."""
        if self.bf16 is None:
            return None
        i = self._index.get(id(p))
        if i is None:
            return None
        if self._shadow_ver < 0 or self.data._version + self._pver != self._shadow_ver:
            self.check_bf16()  # full check only when the cheap one cannot vouch
        return self._shaped(self.bf16, i, p)

    def param_view(self, i: int) -> torch.Tensor:
        return self._shaped(self.data, i, self.params[i])

    def grad_view(self, i: int) -> torch.Tensor:
        return self._shaped(self.grad, i, self.params[i])

    def _flat_like_view(self, i: int, g: torch.Tensor) -> Optional[torch.Tensor]:
        """``g`` as a flat tensor in the arena's element order, when its layout matches
        the arena view's (contiguous, or the same dense channels_last strides)."""
        st = self.strides[i]
        if st is None:
            return g.reshape(-1) if g.is_contiguous() else None
        if tuple(g.stride()) == st:
            return g.as_strided((g.numel(),), (1,))
        return None

    def index_of(self, p: torch.Tensor) -> Optional[int]:
        return self._index.get(id(p))

    def owns_grad(self, i: int) -> bool:
        p = self.params[i]
        g = p.grad
        o, n = self.offsets[i]
        return g is not None and g.data_ptr() == self.grad.data_ptr() + o * 4 and g.numel() == n

    def rebind_grad(self, i: int) -> None:
        """Move a freshly allocated .grad (e.g. after zero_grad(set_to_none=True)) into the arena."""
        p = self.params[i]
        view = self.grad_view(i)
        if p.grad is None:
            view.zero_()
        elif not self.owns_grad(i):
            view.copy_(p.grad)
        p.grad = view

    def rebind_all(self) -> None:
        for i, p in enumerate(self.params):
            o, n = self.offsets[i]
            if p.data.data_ptr() != self.data.data_ptr() + o * 4:
                with torch.no_grad():
                    self._shaped(self.data, i, p).copy_(p.data)
                p.data = self._shaped(self.data, i, p)
        self.gather_grads()

    def gather_grads(self, indices: Optional[Sequence[int]] = None) -> None:
        """Move every non-arena ``.grad`` of ``indices`` (default: all) into the
        arena -- one multi-tensor copy launch on the current stream -- and rebind
        ``.grad`` to the arena views; a missing grad becomes a zero view."""
        idx = range(len(self.params)) if indices is None else indices
        pairs, moved = [], []
        for i in idx:
            p = self.params[i]
            g = p.grad
            if g is None or self.owns_grad(i):
                if g is None:
                    self.rebind_grad(i)
                continue
            flat = self._flat_like_view(i, g) if g.dtype == torch.float32 and g.device == self.device else None
            if flat is None:
                self.rebind_grad(i)
                continue
            o, n = self.offsets[i]
            pairs.append((flat, self.grad[o:o + n]))
            moved.append(i)
        if not pairs:
            return
        if self.device.type == "cuda":
            from ..ops.optim import build_copy_table, multi_copy

            key = tuple(moved) + tuple(s.data_ptr() for s, _ in pairs)
            table = self._tables.get(key)
            if table is None:
                capturing = torch.cuda.is_current_stream_capturing()
                if capturing and self._graph_staging is None:
                    raise RuntimeError("ParamArena: call prepare_graph_capture() before capturing a step")
                # captured: each table takes the next slice of the reserved pinned buffer
                # (a data-parallel step gathers once per bucket, all in one capture)
                off = self._graph_staging_off if capturing else 0
                table = build_copy_table(pairs, staging=self._graph_staging[off:] if capturing else None)
                self._tables[key] = table
                if capturing:
                    self._graph_tables.append((table, self._graph_staging))  # replayed: never evicted
                    self._graph_staging_off = off + table.numel()
                if len(self._tables) > 64:  # address sets are stable under the caching allocator
                    self._tables.popitem(last=False)
            multi_copy(pairs, table=table)
        else:
            with torch.no_grad():
                for s, d in pairs:
                    d.copy_(s)
        for i in moved:
            self.params[i].grad = self.grad_view(i)

    def prepare_graph_capture(self) -> None:
        """Reserve the pinned staging buffer the next captured step's gradient-gather
        table is built in (pinned memory cannot be allocated during a capture)."""
        from ..ops.optim import CHUNK_ELEMS

        rows = sum((n + CHUNK_ELEMS - 1) // CHUNK_ELEMS for _, n in self.offsets)
        self._graph_staging = torch.empty(rows * 4, dtype=torch.int64).pin_memory()
        self._graph_staging_off = 0

    def zero_grad(self) -> None:
        if self.steal_grads:
            for p in self.params:
                p.grad = None
            return
        self.grad.zero_()
        for i, p in enumerate(self.params):
            if not self.owns_grad(i):
                p.grad = self.grad_view(i)

    def is_arena_group(self, params: List[torch.Tensor]) -> bool:
        return len(params) == len(self.params) and all(a is b for a, b in zip(params, self.params))

    def contiguous_range(self, params: List[torch.Tensor]) -> Optional[Tuple[int, int]]:
        """(start, end) in the arena if ``params`` are consecutive arena members, else None."""
        idx = [self.index_of(p) for p in params]
        if any(i is None for i in idx) or not idx:
            return None
        idx_sorted = sorted(idx)
        if idx_sorted != list(range(idx_sorted[0], idx_sorted[-1] + 1)):
            return None
        start = self.offsets[idx_sorted[0]][0]
        last_o, last_n = self.offsets[idx_sorted[-1]]
        end = last_o + last_n
        end = min(self.numel, (end + 3) // 4 * 4)
        return start, end
