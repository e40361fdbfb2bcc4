#!/bin/bash
# Iteration check for MLP-step / Trainer-dispatch changes: the MLP, fused-DP and
# Trainer GPU tests, then the default bench (K = 2000 and the driver's K = 20),
# the phase probe, the 128-256 b32 corner, Trainer.fit via RayAccelerator, and the
# 2-rank shared-GPU bench on the one-launch DP step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/iter}; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_mlp3.py tests/test_comm.py tests/test_trainer.py tests/test_fused_validation.py tests/test_dispatch.py tests/test_ddp_gpu.py \
  -x -v -m gpu -k "not resnet" --timeout 180 --timeout-method thread \
  > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest.log" | head; exit $rc; }
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep -ho '"ms_per_step": [0-9.]*' "$O/$n.log" | sed "s/^/$n /"
}
step bench_one 300 python bench.py --steps 2000 --warmup 200
step bench_one_k20 300 python bench.py --steps 20 --warmup 5
step corner_128_256_b32 300 python bench.py --layer-1 128 --layer-2 256 --batch-size 32
step trainer_ddp 300 python bench.py --via trainer
RLA_BENCH_SHARE_GPU=1 step share2 300 python bench.py --gpus 2 --steps 2000 --warmup 200
timeout -k 10 300 python scripts/mlp_phase_probe.py quick > "$O/phases.log" 2>&1 || { tail -20 "$O/phases.log"; exit 1; }
cat "$O/phases.log" | grep -v amdgpu.ids
grep -h '^{' "$O/trainer_ddp.log" | grep -o '"epoch_split": .*"median_steady_epoch_samples_per_s": [0-9.]*'
# kernel trace of Trainer.fit (worker process included): GPU busy fraction and gaps
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/prof_trainer" -o run -- python3 "$R/bench.py" \
  --via trainer --trainer-epochs 3 > "$O/prof_trainer.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof_trainer.log"; exit 1; }
python scripts/trace_gaps.py "$O/prof_trainer" --pattern mlp3 | tee "$O/trainer_gaps.json"
