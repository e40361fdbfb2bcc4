#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --model resnet50 > gpurun_out/bench_rn50_native.log 2>&1
rc=$?; tail -2 gpurun_out/bench_rn50_native.log; echo "rn50 native rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model resnet50 --impl torch > gpurun_out/bench_rn50_torch.log 2>&1
rc=$?; tail -2 gpurun_out/bench_rn50_torch.log; echo "rn50 torch rc=$rc"
exit $rc
