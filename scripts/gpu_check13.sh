#!/bin/bash
# Rebuilt-tree verification + Trainer-level throughput: full GPU suite, smoke,
# default bench, Trainer.fit bench (RayAccelerator / HorovodRayAccelerator,
# multi-step dispatch vs per-batch), rocprofv3 kernel stats of the bench.
# Every GPU step has its own limit; any failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; O=gpurun_out/r1_c13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo bench failed; tail -20 $O/bench_default.log; exit 1; }
cat $O/bench_default.log
for spd in 64 1; do
  timeout -k 10 300 python scripts/bench_trainer.py --workers 1 --steps-per-dispatch $spd > $O/trainer_ddp_spd$spd.log 2>&1 \
    || { echo "trainer bench spd=$spd failed"; tail -30 $O/trainer_ddp_spd$spd.log; exit 1; }
  tail -c 600 $O/trainer_ddp_spd$spd.log; echo
done
timeout -k 10 300 python scripts/bench_trainer.py --workers 1 --accelerator horovod > $O/trainer_hvd.log 2>&1 \
  || { echo "trainer bench horovod failed"; tail -30 $O/trainer_hvd.log; exit 1; }
tail -c 600 $O/trainer_hvd.log; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 2000 --warmup 200 > $O/prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
