#!/bin/bash
# Trainer-level and Tune-level numbers on the current tree: Trainer.fit through
# RayAccelerator / HorovodRayAccelerator (epoch split), the reference tune_mnist
# sweep (pre-started worker pool), plus the dispatch/validation GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/trainer_tune}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_dispatch.py tests/test_fused_validation.py tests/test_tune.py -x -v -m gpu \
  --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest.log" | head -20; exit $rc; }
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  grep '^{' "$O/$n.log" | cut -c1-400
}
step trainer_ddp 300 python bench.py --via trainer --trainer-epochs 6
step trainer_hvd 300 python bench.py --via trainer --accelerator horovod --trainer-epochs 6
step tune_4x1 600 python scripts/bench_tune.py --trials 4 --workers 1 --epochs 2
echo done
