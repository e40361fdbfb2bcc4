#!/bin/bash
# Native comm-engine self-test (no torch): plain build at world 2 and 4, then the
# host-ASan/UBSan/LSan build at world 2 (device code is not instrumented).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 ./build/comm_selftest 2 > gpurun_out/selftest_w2.log 2>&1 || { echo "plain w2 failed"; tail -20 gpurun_out/selftest_w2.log; exit 1; }
tail -3 gpurun_out/selftest_w2.log
timeout -k 10 180 ./build/comm_selftest 4 > gpurun_out/selftest_w4.log 2>&1 || { echo "plain w4 failed"; tail -20 gpurun_out/selftest_w4.log; exit 1; }
tail -2 gpurun_out/selftest_w4.log
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1:protect_shadow_gap=0
export LSAN_OPTIONS=suppressions=$R/scripts/sanitizers/lsan.supp:print_suppressions=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 300 ./build/comm_selftest_asan 2 > gpurun_out/selftest_asan_w2.log 2>&1
rc=$?; tail -30 gpurun_out/selftest_asan_w2.log; echo "asan rc=$rc"; exit $rc
