#!/bin/bash
# PMC counters of the one-launch fused MNIST step (kind Step1), one rocprofv3 --pmc
# pass per counter group (each under its own hard limit; any failure ends the call),
# then Trainer.fit benches (RayAccelerator / HorovodRayAccelerator, 1 worker,
# full validation + checkpointing) on the current kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_one}; mkdir -p "$O"
B="python bench.py --steps 300 --warmup 30 --graph-steps 0"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS \
  --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || { echo "pass1 rc=$?"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS \
  --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || { echo "pass2 rc=$?"; tail -20 $O/p2.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1 \
  || { echo "pass3 rc=$?"; tail -20 $O/p3.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- $B > $O/p4.log 2>&1 \
  || { echo "pass4 rc=$?"; tail -20 $O/p4.log; exit 1; }
find $O -name "*counter_collection.csv"
timeout -k 10 300 python bench.py --via trainer > "$O/trainer_ddp.log" 2>&1 || { tail -20 "$O/trainer_ddp.log"; exit 1; }
timeout -k 10 300 python bench.py --via trainer --accelerator horovod > "$O/trainer_hvd.log" 2>&1 \
  || { tail -20 "$O/trainer_hvd.log"; exit 1; }
grep -h '^{' "$O"/trainer_*.log | cut -c1-240
# Tune search-space corners (per-GPU batch, layer sizes) on the current kernels
for c in "128 256 128" "128 256 32" "64 128 64" "32 256 32"; do
  set -- $c
  timeout -k 10 300 python bench.py --layer-1 $1 --layer-2 $2 --batch-size $3 > "$O/corner_$1_$2_b$3.log" 2>&1 \
    || { tail -20 "$O/corner_$1_$2_b$3.log"; exit 1; }
done
grep -o '"ms_per_step": [0-9.]*' "$O"/corner_*.log
