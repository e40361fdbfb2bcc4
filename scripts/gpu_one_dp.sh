#!/bin/bash
# One-launch data-parallel step (kind Step1DP): fused-DP correctness tests (2 ranks
# sharing the GPU, batch 64 two-launch and batch 32 one-launch), the MLP kernel
# tests, and the 2-rank shared-GPU bench with the one-launch DP step vs the
# two-launch StepDP (RLA_MLP_ONE_LAUNCH=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/one_dp}; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_comm.py tests/test_mlp3.py -x -v -m gpu \
  -k "fused_dp or dead_peer or mlp3" --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest.log" | head; exit $rc; }
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --warmup 200 > "$O/share2_one.log" 2>&1 \
  || { tail -20 "$O/share2_one.log"; exit 1; }
RLA_MLP_ONE_LAUNCH=0 RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --warmup 200 \
  > "$O/share2_two.log" 2>&1 || { tail -20 "$O/share2_two.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > "$O/bench_one.log" 2>&1 || { tail -20 "$O/bench_one.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O"/share2_*.log "$O"/bench_one.log
grep -h '^\[bench\]' "$O"/share2_*.log | sort | uniq
