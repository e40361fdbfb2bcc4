"""Diagnostic: where does a hipGraph-replayed v3 step diverge from the eager one?

Two engines on the same data: `a` eager, `b` captured with 1 step per graph.
After every step compare params / Adam state / dh1t / h1pre / counters.
"""
import sys

import torch

sys.path.insert(0, '.')
from ray_lightning_accelerators_amd.ops import fused_mlp  # noqa: E402
from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine  # noqa: E402

dev = torch.device('cuda', 0)
g = torch.Generator().manual_seed(5)
x = torch.randint(0, 256, (320, 784), generator=g, dtype=torch.uint8)
y = torch.randint(0, 10, (320,), generator=g)
L1, L2, B = 32, 64, 32
sync_between = len(sys.argv) > 1 and sys.argv[1] == "sync"


def mk():
    e = FusedMLPEngine(L1, L2, B, lr=1e-3, device=dev)
    e.set_data(x, y)
    return e


a, b = mk(), mk()
assert b.capture(1)
a.run(1)
torch.cuda.synchronize()
names = list(fused_mlp.mlp_unpack(a.params, L1, L2).keys())


def report(step):
    torch.cuda.synchronize()
    out = [f"step {step}"]
    pa, pb = fused_mlp.mlp_unpack(a.params, L1, L2), fused_mlp.mlp_unpack(b.params, L1, L2)
    for k in names:
        d = (pa[k] - pb[k]).abs()
        out.append(f"{k}:{d.max().item():.2e}/{(d > 1e-5).float().mean().item():.3f}")
    out.append(f"dh1t:{(a.dh1t.float() - b.dh1t.float()).abs().max().item():.2e}")
    out.append(f"h1pre:{(a.h1pre - b.h1pre).abs().max().item():.2e}")
    out.append(f"xring:{(a.xring.float() - b.xring.float()).abs().max().item():.2e}")
    out.append(f"cnt a{a.counters.tolist()} b{b.counters.tolist()}")
    print(" ".join(out), flush=True)


report(1)
for s in range(2, 14):
    a.step()
    b.step()
    if sync_between:
        torch.cuda.synchronize()
    report(s)
