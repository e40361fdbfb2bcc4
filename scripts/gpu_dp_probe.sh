#!/bin/bash
# Fused data-parallel exchange: correctness tests (2 ranks sharing the GPU) and the
# one-GPU protocol overhead probe for the three protocols (RLA_DP_PROTO):
# granule (default, tagged 8-byte words, no fences), wave (flags, one fencing
# wave per block), all (flags, every wave fences).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/dp}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_comm.py -x -v -m gpu -k "fused_dp or dead_peer or validation" \
  --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for p in granule wave all; do
  RLA_DP_PROTO=$p timeout -k 10 120 python scripts/dp_overhead_probe.py > "$O/probe_$p.log" 2>&1 || { tail -20 "$O/probe_$p.log"; exit 1; }
done
grep us_per_step "$O"/probe_*.log
for p in granule wave; do
  RLA_DP_PROTO=$p RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --warmup 200 > "$O/share2_$p.log" 2>&1 || { tail -20 "$O/share2_$p.log"; exit 1; }
done
grep -o '"ms_per_step": [0-9.]*' "$O"/share2_*.log
