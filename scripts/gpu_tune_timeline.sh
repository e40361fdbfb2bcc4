#!/bin/bash
# Tune sweep (reference tune_mnist, trials x 1 worker, 2 epochs) with the
# cross-process start-up timeline: cold (pool starting with the sweep) and warm.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/tune_tl}; mkdir -p "$O"
for mode in "cold 0 4" "warm 15 8"; do
  set -- $mode
  RLA_TIMELINE="$R/$O/timeline_$1.jsonl" timeout -k 10 600 python scripts/bench_tune.py --trials $3 --workers 1 --epochs 2 \
    --warm $2 > "$O/tune_$1.log" 2>&1 || { echo "tune $1 failed"; tail -30 "$O/tune_$1.log"; exit 1; }
  grep '^{' "$O/tune_$1.log" | cut -c1-330
  python scripts/timeline_report.py "$O/timeline_$1.jsonl" > "$O/timeline_report_$1.txt"
done
