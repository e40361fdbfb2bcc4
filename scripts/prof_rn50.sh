#!/bin/bash
# rocprofv3 kernel traces of ResNet-50 native vs torch (12 steps each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for impl in native torch; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rn50_$impl" -o run -- \
    python3 "$R/bench.py" --model resnet50 --impl $impl --steps 12 --warmup 5 > gpurun_out/prof_rn50_$impl.log 2>&1
  rc=$?; tail -1 gpurun_out/prof_rn50_$impl.log; echo "prof $impl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find gpurun_out/prof_rn50_native gpurun_out/prof_rn50_torch -name "*.csv" | head
