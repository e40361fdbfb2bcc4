#!/bin/bash
# fused BatchNorm+ReLU kernels: numerics tests, then ResNet-50 bench native (fused BN) vs torch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bn.py tests/test_models.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_bn.log | tail -30; tail -3 gpurun_out/pytest_bn.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for impl in native torch; do
  timeout -k 10 300 python bench.py --model resnet50 --impl $impl --steps 30 --warmup 8 > gpurun_out/rn50_${impl}.log 2>&1 || { echo "fail $impl"; tail -20 gpurun_out/rn50_${impl}.log; exit 1; }
  tail -1 gpurun_out/rn50_${impl}.log
done
