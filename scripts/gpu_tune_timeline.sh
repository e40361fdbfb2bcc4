#!/bin/bash
# Tune sweep (reference tune_mnist, 4 trials x 1 worker, 2 epochs) with the
# cross-process start-up timeline, to see where a short trial's time goes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/tune_tl}; mkdir -p "$O"
RLA_TIMELINE="$R/$O/timeline.jsonl" timeout -k 10 600 python scripts/bench_tune.py --trials 4 --workers 1 --epochs 2 \
  > "$O/tune.log" 2>&1 || { echo "tune failed"; tail -30 "$O/tune.log"; exit 1; }
grep '^{' "$O/tune.log" | cut -c1-300
python scripts/timeline_report.py "$O/timeline.jsonl" > "$O/timeline_report.txt"
tail -16 "$O/timeline_report.txt"
