#!/bin/bash
# Multi-step dispatch without host syncs (device slot lists, pinned epoch order,
# graph kept across epochs, deferred logger flush) + chunked two-shot route:
# targeted GPU tests, Trainer-level bench (DDP / Horovod), default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; O=gpurun_out/r1_c14; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dispatch.py tests/test_comm.py tests/test_mlp3.py tests/test_ddp_gpu.py \
  tests/test_native_selftest.py -x -v -m gpu --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -12 $O/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for acc in ddp horovod; do
  timeout -k 10 300 python scripts/bench_trainer.py --workers 1 --accelerator $acc --epochs 4 > $O/trainer_$acc.log 2>&1 \
    || { echo "trainer bench $acc failed"; tail -30 $O/trainer_$acc.log; exit 1; }
  tail -c 900 $O/trainer_$acc.log; echo
done
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo bench failed; tail -20 $O/bench_default.log; exit 1; }
cat $O/bench_default.log
