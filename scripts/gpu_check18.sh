#!/bin/bash
# Current tree: Trainer-level benches with the GC frozen during fit (DDP / Horovod), and the
# Tune sweep (reference tune_mnist example, 4 trials) on one MI355X.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; O=gpurun_out/r1_c18; mkdir -p $O
for acc in ddp horovod; do
  timeout -k 10 300 python scripts/bench_trainer.py --workers 1 --accelerator $acc --epochs 5 > $O/trainer_$acc.log 2>&1 \
    || { echo "trainer bench $acc failed"; tail -30 $O/trainer_$acc.log; exit 1; }
  tail -c 400 $O/trainer_$acc.log; echo
done
timeout -k 10 300 python scripts/bench_trainer.py --workers 1 --batch-size 128 --layer-1 128 --layer-2 256 --epochs 4 \
  > $O/trainer_ddp_128_256_b128.log 2>&1 || { echo "trainer bench big failed"; tail -30 $O/trainer_ddp_128_256_b128.log; exit 1; }
tail -c 400 $O/trainer_ddp_128_256_b128.log; echo
timeout -k 10 600 python scripts/bench_tune.py --trials 4 --workers 1 --epochs 2 > $O/tune.log 2>&1 \
  || { echo "tune bench failed"; tail -30 $O/tune.log; exit 1; }
tail -1 $O/tune.log
timeout -k 10 600 python bench.py --model resnet50 --impl native --steps 20 --warmup 10 > $O/bench_rn50_native.log 2>&1 \
  || { echo "rn50 bench failed"; tail -30 $O/bench_rn50_native.log; exit 1; }
tail -1 $O/bench_rn50_native.log
