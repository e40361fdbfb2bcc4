# the whole GPU suite with device canaries (stray-writer detector), twice
out=gpurun_out/$1
mkdir -p "$out"
for i in 1 2; do
  RLA_CANARY=1 RLA_CANARY_LOG="$out/canary_$i.jsonl" timeout -k 10 500 python -u -m pytest -s -v --timeout 150 --timeout-method thread tests -m gpu > "$out/pytest_gpu_$i.log" 2>&1
  rc=$?; echo "pytest[$i] rc=$rc"; grep -aE "FAILED" "$out/pytest_gpu_$i.log" | head -5; tail -1 "$out/pytest_gpu_$i.log"
  [ -f "$out/canary_$i.jsonl" ] && grep -v fill_after "$out/canary_$i.jsonl" | cut -c1-400 | head -20
  [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
done
exit 0
