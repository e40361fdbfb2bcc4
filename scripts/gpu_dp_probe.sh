#!/bin/bash
# Fused data-parallel exchange: correctness tests (2 ranks sharing the GPU) and the
# one-GPU protocol overhead probe, single-wave fences (default) vs every wave.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/dp}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_comm.py -x -v -m gpu -k "fused_dp or dead_peer or validation" \
  --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/dp_overhead_probe.py > "$O/probe_wave.log" 2>&1 || { tail -20 "$O/probe_wave.log"; exit 1; }
RLA_DP_FENCE=all timeout -k 10 120 python scripts/dp_overhead_probe.py > "$O/probe_all.log" 2>&1 || { tail -20 "$O/probe_all.log"; exit 1; }
grep us_per_step "$O"/probe_*.log
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --warmup 200 > "$O/share2.log" 2>&1 || { tail -20 "$O/share2.log"; exit 1; }
RLA_DP_FENCE=all RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --warmup 200 > "$O/share2_all.log" 2>&1 || { tail -20 "$O/share2_all.log"; exit 1; }
grep -ho '"ms_per_step": [0-9.]*' "$O"/share2*.log
