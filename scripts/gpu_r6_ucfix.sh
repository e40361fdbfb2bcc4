# the uncached-region pool: probe modes 2 (own IPC handle opened / closed each round)
# and 3 (one region kept, the pool), then the GPU suite with the sensitive case repeated
# at the end of the session
out=gpurun_out/$1
mkdir -p "$out"
for m in 3 2; do
  timeout -k 10 100 ./build/uncached_reuse_probe 40 8 $m > "$out/probe_mode$m.log" 2>&1; echo "probe mode $m rc=$?"; tail -1 "$out/probe_mode$m.log"
done
RLA_FIDELITY_REPEAT=30 timeout -k 10 1000 python -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-300 | head -5; tail -1 "$out/pytest_gpu.log"
