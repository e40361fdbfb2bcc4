"""Probe: native RCCL communicator at world size 1 (diagnostics for the _comm engine)."""
import sys
import torch
sys.path.insert(0, '.')
from ray_lightning_accelerators_amd.parallel.comm import native_comm_module  # noqa: E402

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
mod = native_comm_module()
print("module", mod, flush=True)
uid = mod.Communicator.unique_id()
print("uid", len(uid), flush=True)
c = mod.Communicator(0, 1, 0)
print("ctor ok", flush=True)
c.init_rccl(uid)
print("init ok", flush=True)
t = torch.arange(10, device="cuda", dtype=torch.float32)
c.allreduce(t, 0)
torch.cuda.synchronize()
print("allreduce", t.tolist(), c.error_state(), flush=True)
