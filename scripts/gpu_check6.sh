#!/bin/bash
# comm tests + rehearsal of the multi-rank bench path on one GPU (2 ranks share device 0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_comm.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_comm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_comm.log; echo "pytest comm rc=$rc"
[ $rc -eq 0 ] || exit $rc
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 400 --warmup 40 > gpurun_out/bench_share2.log 2>&1
rc=$?; grep -v "NCCL WARN\|^$\|Could not read" gpurun_out/bench_share2.log | tail -4; echo "share2 xgmi rc=$rc"
[ $rc -eq 0 ] || exit $rc
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 400 --warmup 40 --comm torch --graph-steps 0 > gpurun_out/bench_share2_torch.log 2>&1
rc=$?; grep -v "NCCL WARN\|^$\|Could not read" gpurun_out/bench_share2_torch.log | tail -3; echo "share2 gloo rc=$rc"
exit $rc
