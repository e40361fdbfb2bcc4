# A/B: round-4 one-launch kernel (build/base) vs the hooked-prologue + LDS-DMA head pass (tree)
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp3.py -m gpu > "$out/mlp3.log" 2>&1
echo "mlp3 rc=$?"; tail -1 "$out/mlp3.log"
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then d=build/base; else d=.; fi
    (cd $d && timeout -k 10 120 python -u $R/scripts/k20_probe.py --graphs 20 --windows 60) > "$out/k20_${v}_$rep.log" 2>&1 || { echo "k20 $v rc=$?"; exit 1; }
    grep '"graph_steps": 20' "$out/k20_${v}_$rep.log" | cut -c1-200
  done
done
for v in base new; do
  if [ $v = base ]; then d=build/base; else d=.; fi
  (cd $d && timeout -k 10 200 python -u $R/scripts/dp_overhead_probe.py --steps 3000 --worlds 1,8) > "$out/dp_${v}.log" 2>&1 || { echo "dp $v rc=$?"; exit 1; }
  grep -v amdgpu.ids "$out/dp_${v}.log" | cut -c1-220
done
