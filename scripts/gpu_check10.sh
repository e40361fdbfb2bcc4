#!/bin/bash
# arena grad stealing: unit tests, comm/reducer tests, trainer GPU tests, ResNet-50 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena.py tests/test_comm.py tests/test_models.py tests/test_ddp_gpu.py tests/test_native_selftest.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_arena.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_arena.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for impl in native torch; do
  timeout -k 10 300 python bench.py --model resnet50 --impl $impl --steps 30 --warmup 8 > gpurun_out/rn50_${impl}.log 2>&1 || { echo "fail $impl"; tail -20 gpurun_out/rn50_${impl}.log; exit 1; }
  tail -1 gpurun_out/rn50_${impl}.log
done
