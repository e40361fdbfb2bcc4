#!/bin/bash
# Fused MNIST step across the Tune search space's corner configs: bench + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; O=gpurun_out/r1_c20; mkdir -p $O
for cfg in "64 128 64" "128 256 128" "128 256 32"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --layer-1 $1 --layer-2 $2 --batch-size $3 > $O/bench_$1_$2_b$3.log 2>&1 \
    || { echo "bench $cfg failed"; tail -20 $O/bench_$1_$2_b$3.log; exit 1; }
  tail -1 $O/bench_$1_$2_b$3.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --layer-1 128 --layer-2 256 --batch-size 128 --steps 2000 --warmup 200 > $O/prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*stats.csv"
