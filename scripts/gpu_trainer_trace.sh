#!/bin/bash
# Trainer epoch breakdown (train / validation / rest, per-chunk trace) to find the
# slow-epoch stall, plus head/tail phase stamps and default-config kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/trace}; mkdir -p "$O"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep '^{' "$O/$n.log" | cut -c1-300
}
RLA_BENCH_TRACE=1 step trainer_trace 300 python bench.py --via trainer --trainer-epochs 6
step trainer_notrace 300 python bench.py --via trainer --trainer-epochs 6
step phases 300 python scripts/mlp_phase_probe.py
cp gpurun_out/mlp_phases.json "$O/" 2>/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" \
  > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
echo done
