#!/bin/bash
# End-of-round check: the broad round check (full GPU suite, smoke, default bench, N=2
# rehearsals, ResNet-50 DDP sweep), then a rocprofv3 kernel-stats profile of the default
# bench and the driver-shaped bench (K = 20, W = 5).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/final}; mkdir -p "$O"
bash scripts/gpu_round_check.sh "$O" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" \
  > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_default.csv" \;
head -4 "$O/kernel_stats_default.csv" | cut -c1-200
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_k20.log" 2>&1 || { tail -20 "$O/bench_k20.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/bench_k20.log"
