#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels.py -q -m gpu > gpurun_out/pytest_kernels.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_kernels.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mlp_phase_probe.py > gpurun_out/phase.log 2>&1; echo "phase rc=$?"; cat gpurun_out/phase.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; echo "bench rc=$?"; cat gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --graph-steps 0 > gpurun_out/bench_eager.log 2>&1; echo "bench rc=$?"; cat gpurun_out/bench_eager.log
