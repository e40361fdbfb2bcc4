#!/bin/bash
# Implicit host<->device syncs of an in-process Trainer.fit (torchrun, 1 rank) on the fused step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/sync}; mkdir -p "$O"
RLA_SYNC_DEBUG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29545 bench.py --via trainer > "$O/trainer_sync.log" 2>&1 \
  || { tail -20 "$O/trainer_sync.log"; exit 1; }
grep -c "sync-debug" "$O/trainer_sync.log"
grep -A12 "sync-debug" "$O/trainer_sync.log" | head -150
