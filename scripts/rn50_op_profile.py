"""Which framework-level ops launch ResNet-50's small copy / cast / fill kernels:
three fused-path training steps (bs 128) under torch.profiler, aten ops with their
input shapes, sorted by device time (diagnostic for profiles/r3_rn50)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.resnet import resnet50  # noqa: E402
from ray_lightning_accelerators_amd.parallel.arena import ParamArena  # noqa: E402
from ray_lightning_accelerators_amd.parallel.fused_optim import fuse_optimizer  # noqa: E402

dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
model = resnet50(fused_bn=True).to(dev).to(memory_format=torch.channels_last)
arena = ParamArena(model)
opt = fuse_optimizer(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5), arena)
x = torch.randn(128, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (128,), device=dev)


def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(x)
    F.cross_entropy(out.float(), y).backward()
    opt.step()
    opt.zero_grad()


for _ in range(5):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for _ in range(3):
        step()
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_input_shape=True)
print(ka.table(sort_by="self_device_time_total", row_limit=60, max_name_column_width=40,
               max_shapes_column_width=70))
print("\n--- small-kernel sources (aten ops with a copy / cast / fill / add), device us per step")
want = ("aten::copy_", "aten::_to_copy", "aten::clone", "aten::fill_", "aten::zero_", "aten::add", "aten::add_",
        "aten::zeros", "aten::contiguous", "aten::to", "aten::mul_", "aten::mm")
rows = []
for e in ka:
    if e.key in want:
        rows.append((e.device_time_total / 3, e.count // 3, e.key, str(e.input_shapes)[:150]))
for t, n, k, sh in sorted(rows, reverse=True)[:40]:
    print(f"{t:9.1f} {n:4d} {k:18s} {sh}")
