set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/wg1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_wgrad.py > $O/pytest_wgrad.log 2>&1; rc=$?; tail -25 $O/pytest_wgrad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/wgrad_probe.py > $O/wgrad_probe.log 2>&1 || { tail -20 $O/wgrad_probe.log; exit 1; }
cat $O/wgrad_probe.log
timeout -k 10 600 python bench.py --model resnet50 --steps 30 --warmup 10 > $O/rn50.log 2>&1 || { tail -20 $O/rn50.log; exit 1; }
grep '^{' $O/rn50.log | cut -c1-300
