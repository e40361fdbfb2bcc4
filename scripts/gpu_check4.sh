#!/bin/bash
# v3 bring-up: numerics of the pipelined step first (a wrong kernel stops here),
# then the phase probe (v2 vs v3) and the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_mlp3.py -x -q -m gpu > gpurun_out/pytest_mlp3.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_mlp3.log; echo "pytest mlp3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mlp_phase_probe.py > gpurun_out/phase.log 2>&1
rc=$?; cat gpurun_out/phase.log; echo "phase rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; cat gpurun_out/bench_default.log; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests/test_kernels.py -q -m gpu > gpurun_out/pytest_kernels.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_kernels.log; echo "pytest kernels rc=$rc"
exit $rc
