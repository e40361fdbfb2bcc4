#!/bin/bash
# Data-parallel exchange protocols on one GPU: loopback + 2-rank shared-GPU tests,
# then the per-N loopback cost probe.  Each GPU step under its own limit, chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/dp}; mkdir -p "$O"
RLA_FIDELITY_LOG="$R/$O/fidelity.jsonl" timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_mlp3.py tests/test_comm.py -k "loopback or fused_dp or fp32" > "$O/pytest_dp.log" 2>&1
rc=$?; tail -25 "$O/pytest_dp.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dp_overhead_probe.py > "$O/dp_probe.jsonl" 2> "$O/dp_probe.err" || { tail -20 "$O/dp_probe.err"; exit 1; }
cat "$O/dp_probe.jsonl"
