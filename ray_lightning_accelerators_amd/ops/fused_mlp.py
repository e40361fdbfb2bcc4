"""Fused MNIST-classifier MLP step (784 -> L1 -> L2 -> 10).

GPU: one HIP launch per training step (``csrc/mlp_kernels.hip``): forward,
log_softmax + NLL + accuracy, backward and -- at world size 1 -- the Adam
update fused into the weight-gradient epilogues.  CPU: an fp32 PyTorch
reference with identical semantics (also the oracle for the GPU tests).

Parameter arena layout (== ``nn.Linear`` state_dict order of
``layer_1``/``layer_2``/``layer_3``):  W1[L1,784] b1[L1] W2[L2,L1] b2[L2] W3[10,L2] b3[10].
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import require, use_native

IN_FEATURES = 784
NUM_CLASSES = 10
SUPPORTED = {(32, 32), (32, 64), (32, 128), (32, 256), (64, 64), (64, 128), (64, 256),
             (128, 64), (128, 128), (128, 256)}


def mlp_param_count(L1: int, L2: int) -> int:
    return L1 * IN_FEATURES + L1 + L2 * L1 + L2 + NUM_CLASSES * L2 + NUM_CLASSES


def mlp_supported(L1: int, L2: int) -> bool:
    return (int(L1), int(L2)) in SUPPORTED


def mlp_unpack(flat: torch.Tensor, L1: int, L2: int) -> Dict[str, torch.Tensor]:
    """Views of the arena as nn.Linear tensors (state_dict key order)."""
    shapes = [
        ("layer_1.weight", (L1, IN_FEATURES)), ("layer_1.bias", (L1,)),
        ("layer_2.weight", (L2, L1)), ("layer_2.bias", (L2,)),
        ("layer_3.weight", (NUM_CLASSES, L2)), ("layer_3.bias", (NUM_CLASSES,)),
    ]
    out, off = {}, 0
    for name, shp in shapes:
        n = math.prod(shp)
        out[name] = flat[off:off + n].view(shp)
        off += n
    assert off == flat.numel(), "arena size mismatch"
    return out


def _gather_batch(x_u8, x_f32, labels, order, cursor, B, index=None):
    if x_u8 is not None:
        if index is None:
            index = order[cursor * B:(cursor + 1) * B]
        x = x_u8.index_select(0, index).float() / 255.0
        y = labels.index_select(0, index)
    else:
        x = x_f32.reshape(B, IN_FEATURES).float()
        y = labels
    return x, y


def _reference_forward(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    h1 = F.relu(F.linear(x, p["layer_1.weight"], p["layer_1.bias"]))
    h2 = F.relu(F.linear(h1, p["layer_2.weight"], p["layer_2.bias"]))
    return F.linear(h2, p["layer_3.weight"], p["layer_3.bias"])


def mlp_train_step(
    params: torch.Tensor,
    grads: torch.Tensor,
    *,
    L1: int,
    L2: int,
    B: int,
    labels: torch.Tensor,
    x_u8: Optional[torch.Tensor] = None,
    x_f32: Optional[torch.Tensor] = None,
    order: Optional[torch.Tensor] = None,
    counters: Optional[torch.Tensor] = None,
    n_batches: int = 0,
    exp_avg: Optional[torch.Tensor] = None,
    exp_avg_sq: Optional[torch.Tensor] = None,
    stats: Optional[torch.Tensor] = None,
    accumulate_grad: bool = False,
    apply_adam: bool = False,
    advance_step: bool = True,
    lr: float = 1e-3,
    betas: Tuple[float, float] = (0.9, 0.999),
    eps: float = 1e-8,
    weight_decay: float = 0.0,
    lr_tensor: Optional[torch.Tensor] = None,
    adamw: bool = False,
    stamps: Optional[torch.Tensor] = None,
) -> None:
    """One training micro-step of the MNIST MLP over a flat parameter arena.

    u8 mode (``x_u8`` = GPU-resident uint8 dataset [N, 784]): the batch is
    ``order[cursor*B:(cursor+1)*B]`` with ``cursor = counters[1]``, which the
    step advances (mod ``n_batches``) -- so a captured hipGraph replays
    successive batches.  ``counters[0]`` is the optimizer step t.
    """
    if use_native(params):
        require().mlp_train_step(
            x_u8, x_f32, labels, order, counters, int(n_batches), int(B), int(L1), int(L2),
            params, grads, exp_avg, exp_avg_sq, stats, bool(accumulate_grad), bool(apply_adam),
            bool(advance_step), float(lr), float(betas[0]), float(betas[1]), float(eps),
            float(weight_decay), lr_tensor, bool(adamw), stamps,
        )
        return
    # ---- fp32 reference ----
    cursor = int(counters[1].item()) if (counters is not None and x_u8 is not None) else 0
    x, y = _gather_batch(x_u8, x_f32, labels, order, cursor, B)
    with torch.enable_grad():
        leaf = params.detach().clone().requires_grad_(True)
        p = mlp_unpack(leaf, L1, L2)
        logits = _reference_forward(p, x)
        logp = F.log_softmax(logits, dim=1)
        loss = F.nll_loss(logp, y)
        (g,) = torch.autograd.grad(loss, [leaf])
    with torch.no_grad():
        if accumulate_grad:
            g = g + grads
        t = (int(counters[0].item()) if counters is not None else 0) + 1
        if apply_adam:
            from .optim import fused_adam_

            gbuf = g.clone()
            fused_adam_(params, gbuf, exp_avg, exp_avg_sq, lr=lr, betas=betas, eps=eps,
                        weight_decay=weight_decay, adamw=adamw, step=t, lr_tensor=lr_tensor)
        else:
            grads.copy_(g)
        if counters is not None:
            if advance_step:
                counters[0] = t
            if x_u8 is not None:
                counters[1] = (cursor + 1) % n_batches if n_batches > 0 else cursor + 1
        if stats is not None:
            ring = stats.numel() // 4
            slot = (t - 1) % max(ring, 1)
            correct = (logp.argmax(dim=1) == y).sum().float()
            stats.view(-1, 4)[slot] = torch.stack(
                [loss.detach(), correct, torch.tensor(float(B)), torch.tensor(float(t))])


def mlp_shadow_layout(L1: int, L2: int) -> Dict[str, int]:
    """bf16 shadow layout: row-major copy [0, np), W2^T at w2t, W3^T (classes padded to 16) at w3t."""
    np_ = mlp_param_count(L1, L2)
    w2t = (np_ + 7) // 8 * 8
    w3t = w2t + L1 * L2
    return {"np": np_, "w2t": w2t, "w3t": w3t, "total": w3t + 16 * L2}


def mlp_refresh_shadow(params: torch.Tensor, shadow: torch.Tensor, L1: int, L2: int) -> None:
    """Recompute every bf16 shadow from the fp32 master weights."""
    if use_native(params):
        require().mlp_adam(params, params, params, params, shadow, int(L1), int(L2), 0.0, 0.9, 0.999, 1e-8, 0.0,
                           1.0, False, False, None, None)
        return
    lay = mlp_shadow_layout(L1, L2)
    v = mlp_unpack(params, L1, L2)
    with torch.no_grad():
        shadow[: lay["np"]].copy_(params)
        shadow[lay["w2t"]: lay["w3t"]].copy_(v["layer_2.weight"].t().reshape(-1))
        w3t = torch.zeros(L2, 16, dtype=params.dtype, device=params.device)
        w3t[:, :NUM_CLASSES] = v["layer_3.weight"].t()
        shadow[lay["w3t"]: lay["total"]].copy_(w3t.reshape(-1))


MLP3_STEP, MLP3_HEAD, MLP3_TAIL_GRAD, MLP3_TAIL_ADAM, MLP3_PRIME, MLP3_STEP_DP, MLP3_STEP1, MLP3_STEP1_DP = range(8)
ONE_LAUNCH_MAX_B = 32  # MLP3_STEP1 / MLP3_STEP1_DP: one head workgroup
# exchange protocols of MLP3_STEP1_DP (csrc/mlp_step3.hip, "Wave-positioned exchange protocols")
DP_GRANULE, DP_PACKED, DP_OWNER = 0, 1, 2
DP_PROTOS = {"granule": DP_GRANULE, "packed": DP_PACKED, "owner": DP_OWNER}
# floats per (slot, rank) receive area of the packed / owner protocols (comm/xgmi.h kDpUnitAreaFloats)
DP_AREA_FLOATS = 327680


def mlp3_dp_capacity(L1: int, L2: int) -> int:
    """Receive-area capacity (floats) for NativeCommunicator.dp_context that every
    one-launch protocol fits: 2 floats per parameter (granule) or the wave-positioned
    areas (packed / owner)."""
    return max(2 * mlp_param_count(L1, L2), DP_AREA_FLOATS)


def mlp3_hand_words(L1: int, L2: int) -> int:
    """int64 words of the one-launch step's acknowledgement / error buffer (csrc/mlp_step3.hip)."""
    return 32
W1_TILES = IN_FEATURES // 16


def mlp3_h1_copies(L1: int) -> int:
    """H1pre copies per ring slot (csrc/mlp_step3.hip ``H1Copies``): the 49 W1 tiles'
    layer-1 partials are atomically added into ``copies`` separate buffers (tile kt
    into copy kt % copies), which the head sums as it loads them."""
    return 2 if int(L1) <= 64 else 1


def mlp3_buffers(L1: int, L2: int, B: int, device) -> Dict[str, torch.Tensor]:
    """Device scratch of the v3 pipelined step (see csrc/mlp_step3.hip)."""
    bp = (B + 31) // 32 * 32
    return {
        "dh1t": torch.zeros(L1 * bp, dtype=torch.bfloat16, device=device),
        "xring": torch.zeros(2 * W1_TILES * bp * 16, dtype=torch.bfloat16, device=device),
        # 12.20 fixed point (int32): integer atomics make the 49-way split-K sum
        # order-independent; [slot][copy][Bp * L1] (see mlp3_h1_copies)
        "h1pre": torch.zeros(2 * mlp3_h1_copies(L1) * bp * L1, dtype=torch.int32, device=device),
        "act": torch.zeros((L1 + 2 * L2 + 16) * bp, dtype=torch.bfloat16, device=device),
        "yring": torch.full((2 * bp,), -1, dtype=torch.int32, device=device),
        # [0, 5) current state, [5, 10) the head's advanced copy (published by the tail),
        # [10] the one-launch step's launch sequence number (its hand-off tag)
        "counters": torch.zeros(16, dtype=torch.int64, device=device),
        # one-launch step: [0] per-block state acknowledgements (monotonic), [16] wait-timeout flag
        "hand": torch.zeros(mlp3_hand_words(L1, L2), dtype=torch.int64, device=device),
        # per-head-workgroup (sum NLL, #correct, #rows, -) when the batch spans several
        "head_part": torch.zeros(bp // 32 * 4, device=device),
    }


def mlp3_launch(
    kind: int,
    *,
    x_u8: torch.Tensor,
    labels: torch.Tensor,
    order: torch.Tensor,
    counters: torch.Tensor,
    n_batches: int,
    B: int,
    L1: int,
    L2: int,
    params: torch.Tensor,
    grads: torch.Tensor,
    exp_avg: torch.Tensor,
    exp_avg_sq: torch.Tensor,
    shadow: torch.Tensor,
    dh1t: torch.Tensor,
    xring: torch.Tensor,
    h1pre: torch.Tensor,
    act: torch.Tensor,
    yring: torch.Tensor,
    stats: Optional[torch.Tensor] = None,
    advance_step: bool = True,
    lr: float = 1e-3,
    betas: Tuple[float, float] = (0.9, 0.999),
    eps: float = 1e-8,
    weight_decay: float = 0.0,
    grad_scale: float = 1.0,
    lr_tensor: Optional[torch.Tensor] = None,
    adamw: bool = False,
    stamps: Optional[torch.Tensor] = None,
    dp_ctx: Optional[Sequence[int]] = None,
    head_part: Optional[torch.Tensor] = None,
    hand: Optional[torch.Tensor] = None,
    dp_proto: int = -1,
    dp_loop: bool = False,
    repeat: int = 1,
) -> None:
    """One v3 launch (GPU only; ``repeat``: that many identical launches back to back
    from one C++ loop -- every step's state lives on the device).  ``kind``: MLP3_STEP (head + fused tail, world size 1),
    MLP3_HEAD / MLP3_TAIL_GRAD (gradients, before the allreduce), MLP3_TAIL_ADAM
    (Adam with ``grad_scale`` + next-step layer-1 partial, after it), MLP3_PRIME
    (layer-1 pre-activations of the pending batch from the current weights; the
    caller zeroes ``h1pre`` first), MLP3_STEP_DP (head + tail whose Adam epilogue
    sums the gradient tiles of all ranks over xGMI itself; ``dp_ctx`` is
    ``NativeCommunicator.dp_context``), MLP3_STEP1 (the whole step in ONE launch,
    world size 1, B <= 32: every block replays the head's serial chain on its own
    CU and then does its tail share; ``hand`` holds the blocks' acknowledgements), MLP3_STEP1_DP
    (MLP3_STEP1 for world size > 1: each block allreduces its gradient values over xGMI as
    tagged granules between its gradient and its Adam; ``dp_ctx`` as for MLP3_STEP_DP,
    receive area >= 2 floats per parameter for ``dp_proto`` 0).  ``dp_proto``: the
    one-launch exchange -- DP_GRANULE (0, round 2), DP_PACKED (1, one-shot, two values
    per granule), DP_OWNER (2, reduce-scatter / owner Adam / all-gather); -1 reads
    ``RLA_DP_PROTO``.  ``dp_loop``: loopback diagnostic (one process plays every rank of
    ``dp_ctx`` through its own region).  ``order`` is [2, n_batches * B]:
    the current and the next epoch's sample order (counters[4] selects)."""
    require().mlp3(
        int(kind), x_u8, labels, order, counters, int(n_batches), int(B), int(L1), int(L2), params, grads, exp_avg,
        exp_avg_sq, shadow, dh1t, xring, h1pre, act, yring, stats, bool(advance_step), float(lr), float(betas[0]),
        float(betas[1]), float(eps), float(weight_decay), float(grad_scale), lr_tensor, bool(adamw), stamps,
        [int(v) for v in (dp_ctx or ())], head_part, hand, int(dp_proto), bool(dp_loop), int(repeat),
    )


def mlp_adam_(params, grads, exp_avg, exp_avg_sq, shadow, *, L1: int, L2: int, lr: float, step: torch.Tensor,
              betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, grad_scale: float = 1.0,
              adamw: bool = False, lr_tensor: Optional[torch.Tensor] = None) -> None:
    """Adam over the MLP arena (world size > 1, after the allreduce) + shadow refresh."""
    if use_native(params):
        require().mlp_adam(params, grads, exp_avg, exp_avg_sq, shadow, int(L1), int(L2), float(lr), float(betas[0]),
                           float(betas[1]), float(eps), float(weight_decay), float(grad_scale), bool(adamw), True,
                           step, lr_tensor)
        return
    from .optim import fused_adam_

    fused_adam_(params, grads, exp_avg, exp_avg_sq, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                grad_scale=grad_scale, adamw=adamw, step=step, lr_tensor=lr_tensor)
    mlp_refresh_shadow(params, shadow, L1, L2)


def mlp_eval(
    params: torch.Tensor,
    *,
    L1: int,
    L2: int,
    B: int,
    labels: torch.Tensor,
    out: torch.Tensor,
    x_u8: Optional[torch.Tensor] = None,
    x_f32: Optional[torch.Tensor] = None,
    index: Optional[torch.Tensor] = None,
    logits: Optional[torch.Tensor] = None,
) -> None:
    """Forward only.  ``out`` [2]: out[0] += sum NLL, out[1] += #correct.  ``out``
    [ceil(B/32), 2]: per-32-row-chunk (sum NLL, #correct), overwritten -- the GPU
    kernel then runs one workgroup per chunk and the caller's ``out.sum(0)`` is
    deterministic.  Optional log-probs into ``logits``."""
    if use_native(params):
        require().mlp_eval(x_u8, x_f32, labels, index, int(B), int(L1), int(L2), params, logits, out)
        return
    x, y = _gather_batch(x_u8, x_f32, labels, None, 0, B, index=index)
    with torch.no_grad():
        logp = F.log_softmax(_reference_forward(mlp_unpack(params, L1, L2), x), dim=1)
        nll = F.nll_loss(logp, y, reduction="none")
        hit = (logp.argmax(dim=1) == y).float()
        if out.dim() == 2:
            pad = out.size(0) * 32 - B
            out[:, 0] = F.pad(nll, (0, pad)).view(-1, 32).sum(1)
            out[:, 1] = F.pad(hit, (0, pad)).view(-1, 32).sum(1)
        else:
            out[0] += nll.sum()
            out[1] += hit.sum()
        if logits is not None:
            logits.view(B, NUM_CLASSES).copy_(logp)


def init_mlp_params(L1: int, L2: int, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """nn.Linear default init (kaiming_uniform(a=sqrt(5)) == U(+-1/sqrt(fan_in))) into a flat arena."""
    flat = torch.empty(mlp_param_count(L1, L2), dtype=torch.float32)
    views = mlp_unpack(flat, L1, L2)
    fans = {"layer_1": IN_FEATURES, "layer_2": L1, "layer_3": L2}
    for name, t in views.items():
        bound = 1.0 / math.sqrt(fans[name.split(".")[0]])
        t.uniform_(-bound, bound, generator=generator)
    return flat
