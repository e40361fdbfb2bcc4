#!/bin/bash
# ResNet-50 1-GPU: native (arena + fused SGD) vs stock torch at bs 128 / 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for bs in 128 256; do
  for impl in native torch; do
    timeout -k 10 300 python bench.py --model resnet50 --impl $impl --batch-size $bs --steps 30 --warmup 8 > gpurun_out/rn50_${impl}_bs${bs}.log 2>&1 || { echo "fail $impl $bs"; tail -20 gpurun_out/rn50_${impl}_bs${bs}.log; exit 1; }
    tail -1 gpurun_out/rn50_${impl}_bs${bs}.log
  done
done
