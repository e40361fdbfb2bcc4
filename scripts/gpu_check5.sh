#!/bin/bash
# native comm engine bring-up on one MI355X: two ranks share the GPU through IPC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_comm.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_comm.log 2>&1
rc=$?; tail -40 gpurun_out/pytest_comm.log; echo "pytest comm rc=$rc"
exit $rc
