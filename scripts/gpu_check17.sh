#!/bin/bash
# Current-tree verification: full GPU suite, smoke(), default bench, the N>1
# MNIST bench path rehearsed with 2 ranks sharing device 0, and rocprofv3
# kernel stats of the default bench.  Every GPU step has its own limit; any
# failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; O=gpurun_out/r1_c17; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -6 $O/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo bench failed; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29547 bench.py --gpus 2 --steps 1000 --warmup 100 > $O/bench_share2.log 2>&1 \
  || { echo "share2 bench failed"; tail -30 $O/bench_share2.log; exit 1; }
grep metric $O/bench_share2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 2000 --warmup 200 > $O/prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
