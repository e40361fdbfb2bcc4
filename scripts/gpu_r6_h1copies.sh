out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp3.py tests/test_fused_validation.py tests/test_dispatch.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/k20_probe.py --graphs 20 --windows 40 > "$out/k20_$rep.log" 2>&1 || { echo "k20 rc=$?"; exit 1; }
  grep '"graph_steps": 20' $out/k20_$rep.log | cut -c1-160
done
timeout -k 10 120 python -u scripts/dp_phase_probe.py > "$out/phases.log" 2>&1; grep -v amdgpu "$out/phases.log" | cut -c1-420
timeout -k 10 200 python -u scripts/dp_overhead_probe.py --steps 3000 --worlds 1,8 > "$out/dp.log" 2>&1; grep -v amdgpu "$out/dp.log" | cut -c1-200
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_k20.log" 2>&1; tail -1 "$out/bench_k20.log" | cut -c1-200
