"""Debug probe: does the MNIST one-launch step read LDS it never wrote?

Fills the whole LDS of every CU with bf16 +Inf (csrc/debug_tools.hip), then runs
the one-launch fidelity check (tests/test_mlp3.py::test_mlp3_one_launch_grads_vs_fp32_autograd).
A pass right after a plain run and a failure after the poison means a
read-before-write of LDS in the step kernel.

  python scripts/lds_poison_probe.py [--L1 128 --L2 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")


def poison(pattern=0x7F807F80):
    """Every CU's whole LDS (160 KB) set to `pattern` (default: bf16 +Inf pairs)."""
    from ray_lightning_accelerators_amd import ops

    ops.require().lds_poison(pattern, 4096)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L1", type=int, default=128)
    ap.add_argument("--L2", type=int, default=256)
    args = ap.parse_args()
    import test_mlp3 as T

    for label, pre in (("clean", None), ("after_lds_poison", poison), ("clean_again", None),
                       ("after_lds_poison_2", poison)):
        if pre is not None:
            pre()
        try:
            T.test_mlp3_one_launch_grads_vs_fp32_autograd(args.L1, args.L2)
            print(label, "PASS", flush=True)
        except AssertionError as e:
            print(label, "FAIL", str(e)[:300], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
