"""ResNet-50's 1x1 convolutions (bs 128, NHWC bf16): MIOpen (torch conv2d + its
autograd) vs plain GEMMs on the [N*H*W, C] view (fwd / dgrad in bf16, wgrad with
an fp32 output written straight into the fp32 gradient: no zero-fill, no atomics,
no cast).  Prints per-shape microseconds; one JSON line per shape."""
import json
import time

import torch
import torch.nn.functional as F

dev = torch.device("cuda", 0)
N = 128
# (H, Cin, Cout) of every stride-1 1x1 conv in ResNet-50 (conv1 / conv3 of the bottlenecks)
shapes = []
for w, nb, res, first_in in ((64, 3, 56, 64), (128, 4, 28, 256), (256, 6, 14, 512), (512, 3, 7, 1024)):
    for b in range(nb):
        cin = first_in if b == 0 else 4 * w
        rin = res if (b > 0 or w == 64) else res * 2
        shapes.append(("conv1", rin, cin, w))
        shapes.append(("conv3", res, w, 4 * w))
uniq = sorted(set(shapes), key=lambda s: (-s[1], s[2]))


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


tot_m = tot_g = 0.0
for name, H, cin, cout in uniq:
    count = shapes.count((name, H, cin, cout))
    x = torch.randn(N, cin, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = torch.randn(cout, cin, 1, 1, device=dev) * 0.05
    wt = wt.contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, cout, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.detach().requires_grad_()
    wr = wt.detach().requires_grad_()

    def miopen():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = F.conv2d(xr, wr)
        y.backward(dy)

    M = N * H * H
    x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
    dy2 = dy.permute(0, 2, 3, 1).reshape(M, cout)
    w2 = wt.reshape(cout, cin)
    gw = torch.zeros(cout, cin, device=dev)

    def gemm():
        wb = w2.to(torch.bfloat16)
        y = x2 @ wb.t()  # fwd  [M, cout]
        dx = dy2 @ wb  # dgrad [M, cin]
        torch.ops.aten.mm.dtype_out(dy2.t(), x2, torch.float32, out=gw)  # wgrad, fp32
        return y, dx

    # numerics: same results as the conv path (fp32 reference)
    y_ref = F.conv2d(x.float(), wt)
    y_g, dx_g = gemm()
    err = float((y_g.float().reshape(N, H, H, cout) - y_ref.permute(0, 2, 3, 1)).abs().max() / y_ref.abs().max())
    tm, tg = bench(miopen), bench(gemm)
    tot_m += tm * count
    tot_g += tg * count
    print(json.dumps({"shape": [name, H, cin, cout], "count": count, "miopen_us": round(tm, 1),
                      "gemm_us": round(tg, 1), "fwd_rel_err": round(err, 5)}), flush=True)
print(json.dumps({"total_miopen_us": round(tot_m, 1), "total_gemm_us": round(tot_g, 1)}), flush=True)
