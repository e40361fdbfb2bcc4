#!/bin/bash
# Broad current-tree check: full GPU suite, smoke, default bench, N=2 rehearsals
# (actor ranks, torchrun, ResNet-50 DDP with a bucket sweep), MLP gradient error report.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/check}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -x -v -s -m gpu --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest_gpu.log" | head -20; exit $rc; }
grep MLP_FP32_ERR "$O/pytest_gpu.log" > "$O/mlp_fp32_err.log"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep '^{' "$O/$n.log" | cut -c1-260
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
RLA_BENCH_SHARE_GPU=1 step share2_ray 300 python bench.py --gpus 2 --steps 500 --warmup 50
RLA_BENCH_SHARE_GPU=1 step share2_torchrun 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 500 --warmup 50
RLA_BENCH_SHARE_GPU=1 step share2_rn50_sweep 600 python bench.py --gpus 2 --model resnet50 --batch-size 32 \
  --steps 6 --warmup 3 --bucket-sweep 1,4,25
echo done
