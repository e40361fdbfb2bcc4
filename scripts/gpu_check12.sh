#!/bin/bash
# Full GPU suite, then a 2-rank shared-GPU rehearsal of the ResNet-50 DDP bench
# (native: fused BN, arena, C++ reducer over the xGMI two-shot; RCCL unavailable
# with two ranks on one device).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_full.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_full.log | head; exit $rc; }
RLA_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --model resnet50 --batch-size 32 --steps 10 --warmup 3 > gpurun_out/rn50_share2.log 2>&1
rc=$?; grep -E "metric|Error|error" gpurun_out/rn50_share2.log | tail -5; echo "share2 rc=$rc"; exit $rc
