#!/bin/bash
# Trainer-dispatch diagnosis: [RLA_CHUNK_PROBE=1: the engine driven in Trainer-shaped
# chunks (scripts/chunk_probe.py)], the dispatch GPU test, the default bench, and
# Trainer.fit in-process (torchrun, 1 rank) vs on a runtime actor (bench --via trainer).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/chunk}; mkdir -p "$O"
if [ "${RLA_CHUNK_PROBE:-0}" = 1 ]; then
  timeout -k 10 300 python scripts/chunk_probe.py > "$O/chunk_probe.log" 2>&1 || { tail -20 "$O/chunk_probe.log"; exit 1; }
  grep -v amdgpu.ids "$O/chunk_probe.log"
fi
timeout -k 10 300 python -u -m pytest tests/test_dispatch.py tests/test_trainer.py tests/test_fused_validation.py tests/test_checkpoint_writer.py tests/test_ddp_gpu.py -x -q -m gpu \
  --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -20 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > "$O/bench_one.log" 2>&1 || { tail -20 "$O/bench_one.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/bench_one.log"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --via trainer > "$O/trainer_torchrun.log" 2>&1 || { tail -20 "$O/trainer_torchrun.log"; exit 1; }
timeout -k 10 300 python bench.py --via trainer > "$O/trainer_ray.log" 2>&1 || { tail -20 "$O/trainer_ray.log"; exit 1; }
timeout -k 10 300 python bench.py --via trainer --accelerator horovod > "$O/trainer_hvd.log" 2>&1 \
  || { tail -20 "$O/trainer_hvd.log"; exit 1; }
for f in trainer_torchrun trainer_ray trainer_hvd; do
  grep -h '^{' "$O/$f.log" | grep -o '"epoch_split": .*"median_steady_epoch_samples_per_s": [0-9.]*' | sed "s/^/$f /"
done
