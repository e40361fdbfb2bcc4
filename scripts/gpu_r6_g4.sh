# H1pre copies: 2 (tree) vs 4 (build/g4) for L1 <= 64 -- correctness subset, then A/B
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
(cd build/g4 && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp3.py -m gpu -k "pipeline or one_launch_matches or fused_matches or dp_loopback_tracks or h1_copies" -p no:cacheprovider) > "$out/g4_tests.log" 2>&1
rc=$?; echo "g4 tests rc=$rc"; tail -1 "$out/g4_tests.log"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in g2 g4; do
    if [ $v = g4 ]; then d=build/g4; else d=.; fi
    (cd $d && timeout -k 10 120 python -u $R/scripts/k20_probe.py --graphs 20 --windows 60) > "$out/k20_${v}_$rep.log" 2>&1 || { echo "k20 $v rc=$?"; exit 1; }
    echo "$v $(grep '"graph_steps": 20' "$out/k20_${v}_$rep.log" | cut -c1-150)"
  done
done
for v in g2 g4; do
  if [ $v = g4 ]; then d=build/g4; else d=.; fi
  (cd $d && timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5) > "$out/bench_$v.log" 2>&1 || { echo "bench $v rc=$?"; exit 1; }
  echo "$v $(grep '"metric"' "$out/bench_$v.log" | cut -c100-180)"
done
