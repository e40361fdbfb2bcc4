# cross-process corruption detector beside the GPU suite (victim process churning fresh device memory)
out=gpurun_out/$1
mkdir -p "$out"
./build/victim_probe 560 256 16 100 > "$out/victim.jsonl" 2> "$out/victim.err" &
vp=$!
sleep 3
RLA_TEST_CLOCK=1 timeout -k 10 500 python -u -m pytest -v --timeout 150 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$out/pytest_gpu.log"
wait $vp; echo "victim rc=$?"
grep -c '"changed_words"' "$out/victim.jsonl"; head -5 "$out/victim.jsonl" | cut -c1-400; tail -1 "$out/victim.jsonl"
