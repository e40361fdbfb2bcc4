#!/bin/bash
# xGMI two-shot allreduce: kernel + router + reducer tests (ranks share the box's GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_comm.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_comm_ts.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_comm_ts.log; echo "pytest rc=$rc"; exit $rc
