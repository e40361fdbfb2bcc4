# bn_finalize with its epilogue inputs prefetched: BN tests, then ResNet-50 A/B against
# the previous commit (build/base), same box
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bn.py tests/test_conv1x1_stats.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 "$out/tests.log"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then d=build/base; else d=.; fi
    (cd $d && timeout -k 10 300 python -u bench.py --model resnet50 --steps 30 --warmup 10) > "$out/rn50_${v}_$rep.log" 2>&1 || { echo "rn50 $v rc=$?"; exit 1; }
    echo "$v $rep $(grep '"metric"' "$out/rn50_${v}_$rep.log" | cut -c60-150)"
  done
done
