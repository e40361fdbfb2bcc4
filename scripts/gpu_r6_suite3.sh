# the whole GPU suite twice (separate processes, no -x, prints shown), then smoke + default bench
out=gpurun_out/$1
mkdir -p "$out"
for i in 1 2; do
  timeout -k 10 420 python -u -m pytest -s -v --timeout 120 --timeout-method thread tests -m gpu > "$out/pytest_gpu_$i.log" 2>&1
  rc=$?; echo "pytest[$i] rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu_$i.log" | cut -c1-600 | head -8; tail -1 "$out/pytest_gpu_$i.log"
  [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1; echo "smoke rc=$?"; tail -1 "$out/smoke.log"
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_k20.log" 2>&1; echo "bench rc=$?"; tail -1 "$out/bench_k20.log" | cut -c1-300
