"""Which layer of the fused ResNet-50 forward is not bitwise reproducible?  Runs the
same training-mode forward (same weights, same batch, backends already picked) twice
and reports, in forward order, every module whose output differs, with the backend
choices of the convolutions -- one JSON line per differing module, then a summary."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from ray_lightning_accelerators_amd.models.resnet import resnet50  # noqa: E402
from ray_lightning_accelerators_amd.ops import conv as C  # noqa: E402
from ray_lightning_accelerators_amd.parallel.arena import ParamArena  # noqa: E402


def main():
    B = int(os.environ.get("BATCH", "32"))
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    m = resnet50(fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    arena = ParamArena(m)
    arena.enable_bf16_shadow(m)
    g = torch.Generator(device=dev).manual_seed(1)
    xb = torch.randn(B, 3, 224, 224, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    yb = torch.randint(0, 1000, (B,), device=dev, generator=g)
    outs = {}
    order = []

    def hook(name):
        def f(mod, inp, out):
            if isinstance(out, torch.Tensor):
                outs.setdefault(name, []).append(out.detach().clone())
                if name not in order:
                    order.append(name)
        return f

    def step():
        arena.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(xb)
        F.cross_entropy(out.float(), yb).backward()

    step()  # backend picks
    hooks = [mod.register_forward_hook(hook(n)) for n, mod in m.named_modules() if n]
    step()
    step()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    bad = 0
    for n in order:
        a, b = outs[n][0], outs[n][1]
        if not torch.equal(a, b):
            bad += 1
            d = (a.float() - b.float()).abs()
            mod = dict(m.named_modules())[n]
            print(json.dumps({"module": n, "type": type(mod).__name__, "shape": list(a.shape),
                              "max_abs_diff": float(d.max()), "n_diff": int((d > 0).sum()),
                              "numel": a.numel()}), flush=True)
            if bad >= 12:
                break
    print(json.dumps({"modules": len(order), "differing": bad, "batch": B,
                      "first": next((n for n in order if not torch.equal(outs[n][0], outs[n][1])), None),
                      "picks": {k: v["pick"] for k, v in C.choices().items() if k.startswith("fwd")}}), flush=True)


if __name__ == "__main__":
    main()
