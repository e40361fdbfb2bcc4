#!/bin/bash
# Current-tree GPU verification: full `pytest -m gpu`, smoke(), default bench,
# rocprofv3 kernel stats of the default bench.  Usage: scripts/gpu_verify.sh OUTDIR
# Every GPU step runs under its own time limit; any failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/verify}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -4 "$O/pytest_gpu.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > "$O/bench_default.log" 2>&1 || { echo bench failed; tail -20 "$O/bench_default.log"; exit 1; }
grep metric "$O/bench_default.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 2000 --warmup 200 > "$O/prof.log" 2>&1 \
  || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
find "$O/prof" -name "*stats.csv"
