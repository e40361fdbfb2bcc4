#!/bin/bash
# Fused MLP step kernels: numerics tests, per-phase stamps, default + Tune-corner
# benches, rocprofv3 kernel stats of the default and the widest config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/mlp}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_mlp3.py tests/test_kernels.py tests/test_dispatch.py tests/test_fused_validation.py \
  -x -v -m gpu --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$O/pytest.log" | head -20; exit $rc; }
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep '^{' "$O/$n.log" | cut -c1-200
}
step phases 300 python scripts/mlp_phase_probe.py
cp gpurun_out/mlp_phases.json "$O/" 2>/dev/null
grep "B[0-9]" "$O/phases.log" | cut -c1-300
step bench_default 300 python bench.py
for cfg in "128 256 128" "128 256 32" "64 128 64" "32 256 32"; do
  set -- $cfg
  step corner_$1_$2_b$3 300 python bench.py --layer-1 $1 --layer-2 $2 --batch-size $3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_default" -o run -- python3 "$R/bench.py" \
  > "$O/prof_default.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof_default.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_128_256_b32" -o run -- python3 "$R/bench.py" \
  --layer-1 128 --layer-2 256 --batch-size 32 > "$O/prof_wide.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof_wide.log"; exit 1; }
echo done
