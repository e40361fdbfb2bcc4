# the whole GPU suite twice (separate processes, no -x, prints shown), then the fuzzer
out=gpurun_out/$1
mkdir -p "$out"
for i in 1 2; do
  timeout -k 10 420 python -u -m pytest -s -v --timeout 120 --timeout-method thread tests -m gpu > "$out/pytest_gpu_$i.log" 2>&1
  rc=$?; echo "pytest[$i] rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu_$i.log" | cut -c1-400 | head -8; tail -1 "$out/pytest_gpu_$i.log"
  [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
done
timeout -k 10 200 python -u scripts/one_launch_fuzz.py --seconds 120 --out "$out/fuzz.jsonl" > "$out/fuzz.log" 2>&1
echo "fuzz rc=$?"; tail -2 "$out/fuzz.log"
