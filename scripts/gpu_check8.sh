#!/bin/bash
# fused data-parallel tail: comm tests (2 ranks share device 0), mlp3 regression,
# and the 2-rank bench rehearsal with the fused vs. split DP step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_comm.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_comm8.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_comm8.log; echo "pytest comm rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_mlp3.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_mlp3_8.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_mlp3_8.log; echo "pytest mlp3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
for dp in fused split; do
  RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 2000 --warmup 200 --dp $dp \
    > gpurun_out/bench_share2_$dp.log 2>&1
  rc=$?; grep -v "NCCL WARN\|^$\|Could not read" gpurun_out/bench_share2_$dp.log | tail -4; echo "share2 $dp rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
