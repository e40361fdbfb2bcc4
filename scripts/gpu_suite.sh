#!/bin/bash
# Full GPU test suite + smoke + default bench; each GPU step under its own limit,
# chained so that a fault/timeout stops the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_default.log; exit 1; }
cat gpurun_out/bench_default.log
