"""Host-side cost of the eager native ResNet-50 training step (bs 128, bf16): the
bench's model setup (parameter arena, bf16 shadows, fused SGD), 5 warm steps, then
cProfile over 5 steps.  Prints the wall ms/step and the top functions -- tells a
host-bound eager step (Python / library launch overhead) from a device-bound one."""
import cProfile
import io
import pstats
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ray_lightning_accelerators_amd.models.resnet import resnet50  # noqa: E402
from ray_lightning_accelerators_amd.ops.shadow import wants_shadow  # noqa: E402
from ray_lightning_accelerators_amd.parallel.arena import ParamArena  # noqa: E402
from ray_lightning_accelerators_amd.parallel.fused_optim import fuse_optimizer  # noqa: E402

dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
model = resnet50(fused_bn=True).to(dev).to(memory_format=torch.channels_last)
arena = ParamArena(model)
if wants_shadow(model):
    arena.enable_bf16_shadow(model)
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
t0 = time.perf_counter()
for _ in range(5):
    step()
torch.cuda.synchronize()
print(f"eager wall {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms/step", flush=True)
prof = cProfile.Profile()
prof.enable()
t0 = time.perf_counter()
for _ in range(5):
    step()
host = (time.perf_counter() - t0) / 5 * 1e3
torch.cuda.synchronize()
prof.disable()
print(f"host enqueue {host:.2f} ms/step (under cProfile)", flush=True)
buf = io.StringIO()
st = pstats.Stats(prof, stream=buf)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)
print(buf.getvalue())
