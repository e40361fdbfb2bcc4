#!/bin/bash
# Quick kernel A/B: MLP + fused-DP tests, default bench (K = 2000 / 20), 128-256 b32 corner, phase probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/quick}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_mlp3.py tests/test_comm.py -x -q -m gpu -k "mlp3 or fused_dp or dead_peer" \
  --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -20 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep -ho '"ms_per_step": [0-9.]*' "$O/$n.log" | sed "s/^/$n /"
}
step bench_one 300 python bench.py --steps 2000 --warmup 200
step bench_one_b 300 python bench.py --steps 2000 --warmup 200
step bench_one_k20 300 python bench.py --steps 20 --warmup 5
step corner_128_256_b32 300 python bench.py --layer-1 128 --layer-2 256 --batch-size 32
RLA_BENCH_SHARE_GPU=1 step share2 300 python bench.py --gpus 2 --steps 2000 --warmup 200
timeout -k 10 300 python scripts/mlp_phase_probe.py quick > "$O/phases.log" 2>&1 || { tail -20 "$O/phases.log"; exit 1; }
grep -v amdgpu.ids "$O/phases.log"
