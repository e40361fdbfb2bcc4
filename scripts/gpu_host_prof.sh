#!/bin/bash
# Host-side cProfile of an in-process Trainer.fit (torchrun, 1 rank) on the fused step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/hostprof}; mkdir -p "$O"
RLA_BENCH_CPROFILE="$R/$O/cprofile.txt" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --via trainer > "$O/trainer_prof.log" 2>&1 \
  || { tail -20 "$O/trainer_prof.log"; exit 1; }
grep -A75 "ordered by: cumulative\|Ordered by: cumulative" "$O/cprofile.txt" | head -90
