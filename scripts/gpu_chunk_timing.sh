#!/bin/bash
# Per-chunk host vs GPU time of an in-process Trainer.fit (RLA_CHUNK_TIMING=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/ctiming}; mkdir -p "$O"
RLA_CHUNK_TIMING=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29546 bench.py --via trainer > "$O/trainer_timing.log" 2>&1 \
  || { tail -20 "$O/trainer_timing.log"; exit 1; }
grep "chunk-timing" "$O/trainer_timing.log"
grep -h '^{' "$O/trainer_timing.log" | grep -o '"epoch_split": .*"median_steady_epoch_samples_per_s": [0-9.]*'
