#!/bin/bash
# First GPU bring-up: kernel numerics, bench (native vs stock torch), rocprof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== host: $(hostname) gpus: $(python -c 'import torch;print(torch.cuda.device_count())')"
timeout -k 10 900 python -m pytest tests/test_kernels.py -q -m gpu > gpurun_out/pytest_kernels.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_kernels.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_native.log 2>&1; rc=$?; cat gpurun_out/bench_native.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --graph-steps 0 > gpurun_out/bench_native_eager.log 2>&1; rc=$?; cat gpurun_out/bench_native_eager.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --impl torch > gpurun_out/bench_torch.log 2>&1; rc=$?; cat gpurun_out/bench_torch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_native" -o run -- python3 "$R/bench.py" --steps 500 --warmup 50 --graph-steps 0 > gpurun_out/prof_native.log 2>&1; rc=$?; tail -3 gpurun_out/prof_native.log; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_torch" -o run -- python3 "$R/bench.py" --steps 300 --warmup 30 --impl torch > gpurun_out/prof_torch.log 2>&1; rc=$?; echo "prof torch rc=$rc"
find gpurun_out -name "*stats*.csv" | head
