"""Device time of the fused 1x1 input gradient + BatchNorm backward partial
(csrc/conv1x1.hip BWD) at ResNet-50's identity-block shapes (bs 128)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
for m, k, n in [(128 * 56 * 56, 64, 256), (128 * 28 * 28, 128, 512)]:
    dy1 = torch.randn(m, k, device=dev).to(torch.bfloat16)
    wt = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    dy2, yb, xb = (torch.randn(m, n, device=dev).to(torch.bfloat16) for _ in range(3))
    f = lambda: ops.require().conv1x1_bn_bwd(dy1, wt, dy2, yb, xb)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1_000_000)
    s.record()
    for _ in range(20):
        f()
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) * 1e3 / 20
    gb = (m * k + 4 * m * n) * 2 / 1e9
    print(json.dumps({"M": m, "K": k, "N": n, "us": round(us, 1), "TBps": round(gb / us * 1e6 / 1e3, 2)}), flush=True)
