#!/bin/bash
# One-launch fused MNIST step: bitwise tests vs head + tail, phase stamps of both
# forms, default bench one-launch vs two-launch (RLA_MLP_ONE_LAUNCH=0), kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/one}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_mlp3.py -x -v -m gpu --timeout 120 --timeout-method thread \
  > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$O/pytest.log" | head -20; exit $rc; }
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep '^{' "$O/$n.log" | cut -c1-240
}
step phases 300 python scripts/mlp_phase_probe.py
cp gpurun_out/mlp_phases.json "$O/" 2>/dev/null
grep "B[0-9]" "$O/phases.log" | cut -c1-300
step bench_one 300 python bench.py
step bench_one_k20 120 python bench.py --steps 20 --warmup 5
RLA_MLP_ONE_LAUNCH=0 step bench_two 300 python bench.py
step corner_128_256_b32 300 python bench.py --layer-1 128 --layer-2 256 --batch-size 32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_default" -o run -- python3 "$R/bench.py" \
  > "$O/prof_default.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof_default.log"; exit 1; }
echo done
