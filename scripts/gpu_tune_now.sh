#!/bin/bash
# Tune sweeps on the current tree: reference tune_mnist (4 trials x 1 worker, 2 epochs)
# cold, and config 4 (4 trials x RayAccelerator(num_workers=2)) on a virtual 8-GPU ledger.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/tune_now}; mkdir -p "$O"
timeout -k 10 600 python scripts/bench_tune.py --trials 4 --workers 1 --epochs 2 > "$O/tune_cold.log" 2>&1 \
  || { tail -30 "$O/tune_cold.log"; exit 1; }
grep '^{' "$O/tune_cold.log" | cut -c1-330
timeout -k 10 600 python scripts/bench_tune.py --trials 4 --workers 2 --epochs 2 --share-gpu 8 --warm 15 \
  > "$O/tune_cfg4_share.log" 2>&1 || { tail -30 "$O/tune_cfg4_share.log"; exit 1; }
grep '^{' "$O/tune_cfg4_share.log" | cut -c1-330
