"""Per-shape device time of ResNet-50's stride-1 1x1 forward convolutions at batch 128
(bf16, NHWC) followed by the BatchNorm partial sums of their output: the MFMA
kernel that sums in its epilogue (csrc/conv1x1.hip) against hipBLASLt / MIOpen +
the separate partial pass.  One JSON line per (shape, arm)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_lightning_accelerators_amd import ops  # noqa: E402
from ray_lightning_accelerators_amd.ops.conv import _bn_partial, _from2d, _time, conv1x1_stats_hip  # noqa: E402

B = int(os.environ.get("BATCH", "128"))
# (H = W, Cin, Cout): conv1 / conv3 / stride-1 downsample of every stage
SHAPES = [
    (56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128),
    (28, 128, 512), (28, 512, 128), (28, 512, 256),
    (14, 256, 1024), (14, 1024, 256), (14, 1024, 512),
    (7, 512, 2048), (7, 2048, 512),
]
REPS = 20


def main():
    torch.backends.cudnn.benchmark = True  # MIOpen find, as the ResNet-50 bench runs it
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    conv = torch.ops.aten.convolution
    for hw, cin, cout in SHAPES:
        x = torch.randn(B, cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wb = (torch.randn(cout, cin, device=dev) / cin ** 0.5).to(torch.bfloat16)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        w4 = wb.view(cout, cin, 1, 1)
        y, part = conv1x1_stats_hip(x, wb)
        ref = torch.mm(x2, wb.t())
        err = float((y.permute(0, 2, 3, 1).reshape(-1, cout).float() - ref.float()).norm() / ref.float().norm())
        arms = {
            "hip_stats": lambda: conv1x1_stats_hip(x, wb),
            "gemm": lambda: torch.mm(x2, wb.t()),
            "gemm+partial": lambda: _bn_partial(_from2d(torch.mm(x2, wb.t()), B, hw, hw)),
            "miopen": lambda: conv(x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1),
            "miopen+partial": lambda: _bn_partial(conv(x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)),
        }
        m = B * hw * hw
        mb = (m * cin + m * cout + cin * cout) * 2 / 1e6
        for name, fn in arms.items():
            t = min(_time(fn, REPS), _time(fn, REPS)) * 1e3 / REPS
            print(json.dumps({"hw": hw, "cin": cin, "cout": cout, "batch": B, "arm": name, "us": round(t, 1),
                              "gemm_min_MB": round(mb, 1), "TBps_min": round(mb / t / 1e0, 2) if t else None,
                              "rel_err_vs_gemm": round(err, 6)}), flush=True)
    ops.require()


if __name__ == "__main__":
    main()
