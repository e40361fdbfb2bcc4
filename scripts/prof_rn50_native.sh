#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rn50_fbn" -o run -- \
  python3 "$R/bench.py" --model resnet50 --impl native --steps 12 --warmup 5 > gpurun_out/prof_rn50_fbn.log 2>&1
rc=$?; tail -1 gpurun_out/prof_rn50_fbn.log; echo "rc=$rc"; exit $rc
