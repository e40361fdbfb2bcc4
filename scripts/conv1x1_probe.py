"""ResNet-50's stride-1 1x1 convolutions (bs 128, NHWC bf16), per operation:
MIOpen (aten convolution / convolution_backward) vs plain GEMMs on the [N*H*W, C]
views -- forward and dgrad in bf16, wgrad with an fp32 output (what the fp32
gradient needs: MIOpen's bf16 wgrad is followed by a cast).  One JSON line per
shape with microseconds per op and backend."""
import json
import time

import torch

dev = torch.device("cuda", 0)
N = 128
shapes = []
for w, nb, res, first_in in ((64, 3, 56, 64), (128, 4, 28, 256), (256, 6, 14, 512), (512, 3, 7, 1024)):
    for b in range(nb):
        cin = first_in if b == 0 else 4 * w
        rin = res if (b > 0 or w == 64) else res * 2
        shapes.append((rin, cin, w))
        shapes.append((res, w, 4 * w))
uniq = sorted(set(shapes), key=lambda s: (-s[0], s[1]))


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


tot = {"miopen": 0.0, "gemm": 0.0, "best": 0.0}
for H, cin, cout in uniq:
    count = shapes.count((H, cin, cout))
    x = torch.randn(N, cin, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, cout, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = N * H * H
    x2, dy2, w2 = x.permute(0, 2, 3, 1).reshape(M, cin), dy.permute(0, 2, 3, 1).reshape(M, cout), wb.reshape(cout, cin)
    gw = torch.zeros(cout, cin, device=dev)
    conv = torch.ops.aten.convolution
    cbw = torch.ops.aten.convolution_backward
    ops = {
        "fwd": {"miopen": lambda: conv(x, wb, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1),
                "gemm": lambda: x2 @ w2.t()},
        "dgrad": {"miopen": lambda: cbw(dy, x, wb, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                        [True, False, False]),
                  "gemm": lambda: dy2 @ w2},
        "wgrad": {"miopen": lambda: cbw(dy, x, wb, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                        [False, True, False])[1].float(),
                  "gemm": lambda: torch.ops.aten.mm.dtype_out(dy2.t(), x2, torch.float32, out=gw)},
    }
    row = {"shape": [H, cin, cout], "count": count}
    for op, cands in ops.items():
        t = {k: round(bench(f), 1) for k, f in cands.items()}
        row[op] = t
        tot["miopen"] += t["miopen"] * count
        tot["gemm"] += t["gemm"] * count
        tot["best"] += min(t.values()) * count
    # numerics of the gemm path against an fp32 reference
    ref = x.float().permute(0, 2, 3, 1).reshape(M, cin) @ w2.float().t()
    row["fwd_rel_err"] = round(float(((x2 @ w2.t()).float() - ref).abs().max() / ref.abs().max()), 5)
    print(json.dumps(row), flush=True)
print(json.dumps({k + "_us_per_step": round(v, 1) for k, v in tot.items()}), flush=True)
