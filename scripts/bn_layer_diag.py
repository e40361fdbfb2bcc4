"""Per-layer error of the fused-BN ResNet-50 (bf16) vs the stock-BN model (bf16),
both against an fp32 reference with identical weights (GPU diagnostic)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_lightning_accelerators_amd.models.resnet import resnet50  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    a = resnet50(10, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    b = resnet50(10, fused_bn=False).to(dev).to(memory_format=torch.channels_last)
    r = resnet50(10, fused_bn=False).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    r.load_state_dict(a.state_dict())
    x = torch.randn(16, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    outs = {}

    def grab(tag):
        def hook(mod, inp, out):
            outs.setdefault(tag, []).append(out.detach().float())
        return hook

    for tag, m in (("a", a), ("b", b), ("r", r)):
        for name, sub in m.named_modules():
            if name.endswith("bn1") or name.endswith("bn2") or name.endswith("bn3") or name.endswith("downsample"):
                sub.register_forward_hook(grab(tag))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        la = a(x)
        lb = b(x)
    lr = r(x)
    names = [n for n, s in r.named_modules() if n.endswith(("bn1", "bn2", "bn3", "downsample"))]
    for i, n in enumerate(names):
        ra = outs["r"][i]
        # stock bn outputs are pre-activation: compare after the same activation as the fused module
        ea = (outs["a"][i] - (F.relu(ra) if "downsample" not in n and not n.endswith("bn3") else ra)).norm() / ra.norm()
        eb = (outs["b"][i] - ra).norm() / ra.norm()
        print(f"{n:28s} fused {float(ea):.4f}  stock {float(eb):.4f}  mean|r| {float(ra.abs().mean()):.3f}")
    print("logits rel err fused", float((la.float() - lr).norm() / lr.norm()), "stock",
          float((lb.float() - lr).norm() / lr.norm()))


if __name__ == "__main__":
    main()
