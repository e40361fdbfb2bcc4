"""Fuse a user's torch optimizer onto the flat arena without replacing it.

``configure_optimizers`` returns a stock ``torch.optim.Adam``/``AdamW``/``SGD``
(reference workloads).  Rather than swapping the object (LR
schedulers keep a reference to it), :func:`fuse_optimizer` rebinds its
``step``/``zero_grad`` to ONE gfx950 launch per param group over the arena
slice the group covers.  Optimizer state lives in arena-shaped buffers and is
exposed through ``optimizer.state[p]`` as per-parameter views, so
``optimizer.state_dict()`` keeps torch's exact format (Lightning checkpoint
``optimizer_states``).
"""
from __future__ import annotations

import types
from typing import Callable, List, Optional

import torch

from ..ops.optim import fused_adam_, fused_sgd_
from .arena import ParamArena

SUPPORTED = (torch.optim.Adam, torch.optim.AdamW, torch.optim.SGD)


def can_fuse(opt: torch.optim.Optimizer, arena: ParamArena) -> bool:
    if type(opt) not in SUPPORTED:
        return False
    for g in opt.param_groups:
        if g.get("amsgrad") or g.get("differentiable"):
            return False
        if arena.contiguous_range(g["params"]) is None:
            return False
        if isinstance(opt, torch.optim.SGD) and g.get("momentum", 0) == 0 and g.get("dampening", 0) != 0:
            return False
    return True


class _GroupState:
    def __init__(self, arena: ParamArena, start: int, end: int, kind: str):
        self.start, self.end = start, end
        self.kind = kind
        n = end - start
        dev = arena.device
        if kind == "adam":
            self.m = torch.zeros(n, device=dev)
            self.v = torch.zeros(n, device=dev)
        else:
            self.buf = torch.zeros(n, device=dev)
        self.step = 0
        # device scalars (enable_device_scalars): the step counter and learning rate
        # the kernel reads at run time, so one captured step replays correctly
        self.step_t: Optional[torch.Tensor] = None
        self.lr_t: Optional[torch.Tensor] = None
        self.lr_host: Optional[float] = None

    def sync_lr(self, lr: float) -> None:
        """Refresh the device learning rate when the host value changed (a scheduler
        step): one fill kernel, stream-ordered before the next step."""
        if self.lr_t is not None and lr != self.lr_host:
            self.lr_t.fill_(lr)
            self.lr_host = lr


def fuse_optimizer(opt: torch.optim.Optimizer, arena: ParamArena,
                   grad_scale_fn: Optional[Callable[[], float]] = None) -> torch.optim.Optimizer:
    """Rebind ``opt.step`` / ``opt.zero_grad`` to fused arena kernels (in place)."""
    if not can_fuse(opt, arena):
        return opt
    kind = "sgd" if isinstance(opt, torch.optim.SGD) else "adam"
    adamw = isinstance(opt, torch.optim.AdamW)
    groups: List[_GroupState] = []
    for g in opt.param_groups:
        s, e = arena.contiguous_range(g["params"])
        gs = _GroupState(arena, s, e, kind)
        groups.append(gs)
        # expose per-param views in torch's state layout
        for p in g["params"]:
            i = arena.index_of(p)
            if kind == "adam":
                opt.state[p] = {"step": torch.tensor(0.0),
                                "exp_avg": arena.shaped_slice(gs.m, i, s),
                                "exp_avg_sq": arena.shaped_slice(gs.v, i, s)}
            elif g.get("momentum", 0) != 0:
                opt.state[p] = {"momentum_buffer": arena.shaped_slice(gs.buf, i, s)}

    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        scale = grad_scale_fn() if grad_scale_fn is not None else 1.0
        arena.rebind_all()
        for g, gs in zip(self.param_groups, groups):
            p = arena.data[gs.start:gs.end]
            gr = arena.grad[gs.start:gs.end]
            gs.step += 1
            step, lr_t = gs.step, None
            if gs.step_t is not None:
                # device scalars: the counter advances on the stream (inside a captured
                # step too), the kernel reads it and the learning rate at run time
                if gs.step_t.device.type != "cuda" or not torch.cuda.is_current_stream_capturing():
                    gs.sync_lr(float(g["lr"]))
                gs.step_t.add_(1)
                # (CPU: never captured -- the host value, in the reference's double precision)
                step, lr_t = gs.step_t, (gs.lr_t if gs.lr_t.is_cuda else None)
            if gs.kind == "adam":
                b1, b2 = g["betas"]
                fused_adam_(p, gr, gs.m, gs.v, lr=float(g["lr"]), betas=(b1, b2), eps=g["eps"],
                            weight_decay=g["weight_decay"], grad_scale=scale, adamw=adamw,
                            maximize=g.get("maximize", False), step=step, lr_tensor=lr_t)
                for q in g["params"]:
                    st = self.state.get(q)
                    if st is not None and "step" in st:
                        st["step"].fill_(float(gs.step))
            else:
                fused_sgd_(p, gr, gs.buf if g.get("momentum", 0) != 0 else None, lr=float(g["lr"]),
                           momentum=g.get("momentum", 0.0), dampening=g.get("dampening", 0.0),
                           weight_decay=g.get("weight_decay", 0.0), nesterov=g.get("nesterov", False),
                           maximize=g.get("maximize", False), grad_scale=scale, step=step, lr_tensor=lr_t,
                           p_bf16=arena.bf16[gs.start:gs.end] if arena.bf16 is not None else None)
            if gs.kind == "adam" and arena.bf16 is not None:
                arena.bf16[gs.start:gs.end].copy_(p)  # Adam path: shadow refreshed by one cast
        return loss

    def zero_grad(self, set_to_none: bool = True):
        arena.zero_grad()

    orig_load = opt.load_state_dict

    def load_state_dict(self, state_dict):
        orig_load(state_dict)
        # torch replaced the state tensors: copy them back into the arena buffers
        for g, gs in zip(self.param_groups, groups):
            for p in g["params"]:
                st = self.state.get(p, {})
                i = arena.index_of(p)
                if gs.kind == "adam" and "exp_avg" in st:
                    m_v = arena.shaped_slice(gs.m, i, gs.start)
                    v_v = arena.shaped_slice(gs.v, i, gs.start)
                    m_v.copy_(st["exp_avg"].reshape(p.shape))
                    v_v.copy_(st["exp_avg_sq"].reshape(p.shape))
                    gs.step = int(float(st.get("step", 0)))
                    self.state[p] = {"step": torch.tensor(float(gs.step)), "exp_avg": m_v, "exp_avg_sq": v_v}
                elif gs.kind == "sgd" and "momentum_buffer" in st and st["momentum_buffer"] is not None:
                    b_v = arena.shaped_slice(gs.buf, i, gs.start)
                    b_v.copy_(st["momentum_buffer"].reshape(p.shape))
                    gs.step = max(gs.step, 1)
                    self.state[p] = {"momentum_buffer": b_v}
        for gs in groups:
            if gs.step_t is not None:
                gs.step_t.fill_(gs.step)

    def enable_device_scalars(self):
        """Step counter and learning rate as device scalars (graph-captured steps:
        ``lightning/graph_step.py``).  The host ``step`` keeps counting too."""
        for g, gs in zip(self.param_groups, groups):
            if gs.step_t is None:
                gs.step_t = torch.full((1,), gs.step, dtype=torch.int64, device=arena.device)
                gs.lr_t = torch.full((1,), float(g["lr"]), dtype=torch.float32, device=arena.device)
                gs.lr_host = float(g["lr"])

    def sync_host_state(self):
        """Per-parameter ``state[p]["step"]`` (Adam) from the host counters, which a
        graph replay advances without touching the per-parameter tensors."""
        for g, gs in zip(self.param_groups, groups):
            if gs.kind != "adam":
                continue
            for q in g["params"]:
                st = self.state.get(q)
                if st is not None and "step" in st and float(st["step"]) != float(gs.step):
                    st["step"].fill_(float(gs.step))

    # keep torch's LR-scheduler bookkeeping happy (it wraps optimizer.step)
    step._wrapped_by_lr_sched = True
    orig_step_fn = step

    def counted_step(self, closure=None):
        self._opt_called = True
        return orig_step_fn(self, closure)

    counted_step._wrapped_by_lr_sched = True
    opt.step = types.MethodType(counted_step, opt)
    opt.zero_grad = types.MethodType(zero_grad, opt)
    opt.load_state_dict = types.MethodType(load_state_dict, opt)
    opt.enable_device_scalars = types.MethodType(enable_device_scalars, opt)
    opt.sync_host_state = types.MethodType(sync_host_state, opt)
    opt._rla_fused = True
    opt._rla_groups = groups
    return opt
