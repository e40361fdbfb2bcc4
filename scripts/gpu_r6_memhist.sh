# the GPU suite with allocator history on (RLA_MEMHIST=1): a fidelity failure's
# post-mortem then names the previous owners of the corrupted range
out=gpurun_out/$1
mkdir -p "$out"
RLA_MEMHIST=1 timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-300 | head -8; tail -1 "$out/pytest_gpu.log"
