# round 6: cross-XCD coherence probe, then the whole GPU suite without -x (diagnostics on)
out=gpurun_out/$1
mkdir -p "$out"
for m in 0 1 2 3; do
  timeout -k 10 90 ./build/coherence_probe $m 1000 2048 >> "$out/coherence.jsonl" 2>&1 || { echo "probe mode $m rc=$?"; exit 1; }
done
cat "$out/coherence.jsonl"
timeout -k 10 900 python -u -m pytest -v -rA --timeout 120 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
echo "pytest rc=$?"; grep -E "FAILED|ERROR|FIRST_BAD|XPASS|xfail" "$out/pytest_gpu.log" | head -20; tail -2 "$out/pytest_gpu.log"
