#!/bin/bash
# New bench modes + the tests that cover them: fused validation, xGMI validation
# fallback, self-launched ranks, torch-graph stock baseline, Trainer-level number.
# Usage: scripts/gpu_bench_modes.sh OUTDIR.  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/modes}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_mlp3.py tests/test_fused_validation.py tests/test_bench.py tests/test_comm.py -x -v -m gpu \
  --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -4 "$O/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest.log" | head -20; exit $rc; }
step() {  # name, limit, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep '^{' "$O/$n.log" | cut -c1-600
}
step bench_torch_graph 300 python bench.py --impl torch-graph --steps 2000 --warmup 200
step bench_torch 300 python bench.py --impl torch --steps 1000 --warmup 100
step bench_native 300 python bench.py --steps 2000 --warmup 200
step trainer_n1 300 python bench.py --via trainer --trainer-epochs 5
step trainer_hvd_n1 300 python bench.py --via trainer --accelerator horovod --trainer-epochs 5
RLA_BENCH_SHARE_GPU=1 step share2_ray 300 python bench.py --gpus 2 --steps 500 --warmup 50
RLA_BENCH_SHARE_GPU=1 step share2_torchrun 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 50
RLA_BENCH_SHARE_GPU=1 step share2_hvd 300 python bench.py --gpus 2 --accelerator horovod --steps 500 --warmup 50
RLA_BENCH_SHARE_GPU=1 step share2_trainer 300 python bench.py --gpus 2 --via trainer --trainer-epochs 3
for cfg in "128 256 128" "128 256 32" "64 128 64"; do
  set -- $cfg
  step corner_$1_$2_b$3 300 python bench.py --layer-1 $1 --layer-2 $2 --batch-size $3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_128_256_b128" -o run -- \
  python3 "$R/bench.py" --layer-1 128 --layer-2 256 --batch-size 128 > "$O/prof_128.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof_128.log"; exit 1; }
echo done
