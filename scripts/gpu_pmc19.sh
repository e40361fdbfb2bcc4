#!/bin/bash
# PMC counters of the fused MNIST step (head + tail kernels), one pass per
# counter group, each under its own hard limit; any failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; O=gpurun_out/r1_pmc; mkdir -p $O
B="python bench.py --steps 300 --warmup 30 --graph-steps 0"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS \
  --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || { echo "pass1 rc=$?"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS \
  --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || { echo "pass2 rc=$?"; tail -20 $O/p2.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1 \
  || { echo "pass3 rc=$?"; tail -20 $O/p3.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- $B > $O/p4.log 2>&1 \
  || { echo "pass4 rc=$?"; tail -20 $O/p4.log; exit 1; }
find $O -name "*counter_collection.csv" | head
