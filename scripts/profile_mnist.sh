#!/bin/bash
# rocprofv3 kernel statistics of the headline step (v3 fused MNIST) and of the
# ResNet-50 arena path; summaries land in gpurun_out/prof_* (copy to profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_v3" -o run -- \
  python3 "$R/bench.py" --steps 2000 --warmup 100 > gpurun_out/prof_v3.log 2>&1
rc=$?; tail -1 gpurun_out/prof_v3.log; echo "prof v3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rn50" -o run -- \
  python3 "$R/bench.py" --model resnet50 --steps 10 --warmup 3 > gpurun_out/prof_rn50.log 2>&1
rc=$?; tail -1 gpurun_out/prof_rn50.log; echo "prof rn50 rc=$rc"
find gpurun_out/prof_v3 gpurun_out/prof_rn50 -name "*kernel_stats.csv"
exit $rc
