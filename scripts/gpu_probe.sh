#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 5 60 ./scripts/probes/tr_probe > gpurun_out/tr_probe.log 2>&1; echo "probe rc=$?"
timeout -k 10 600 python -m pytest tests/test_kernels.py -q -m gpu > gpurun_out/pytest_kernels.log 2>&1; echo "pytest rc=$?"
tail -30 gpurun_out/pytest_kernels.log
