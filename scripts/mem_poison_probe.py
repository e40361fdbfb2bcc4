"""Debug probe: does the MNIST one-launch step read device memory it never wrote?

Fills the caching allocator's free blocks with +Inf (many small and large tensors
allocated, filled, freed), so the engine's later allocations reuse them, then runs
the one-launch fidelity check for both model sizes.  A failure only after the poison
means a read of memory that torch.empty-style allocation does not initialise.

  python scripts/mem_poison_probe.py
"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")


def poison(fill=float("inf")):
    dev = torch.device("cuda", 0)
    keep = []
    for size in [256, 4096, 65536, 1 << 20, 1 << 22] * 40 + [1 << 26] * 8:
        keep.append(torch.full((size // 4,), fill, device=dev))
    torch.cuda.synchronize()
    del keep  # blocks go back to torch's cache, still holding Inf


def main():
    import test_mlp3 as T

    for label, pre in (("clean", None), ("after_mem_poison", poison)):
        for L1, L2 in ((32, 64), (128, 256)):
            if pre is not None:
                pre()
            try:
                T.test_mlp3_one_launch_grads_vs_fp32_autograd(L1, L2)
                print(label, L1, L2, "PASS", flush=True)
            except AssertionError as e:
                print(label, L1, L2, "FAIL", str(e)[:300], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
