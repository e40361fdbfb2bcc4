# the GPU suite with allocator history, then the 128-256 fidelity case 25 more times in
# the same session (RLA_FIDELITY_REPEAT), no -x
out=gpurun_out/$1
mkdir -p "$out"
RLA_MEMHIST=1 RLA_FIDELITY_REPEAT=40 timeout -k 10 1000 python -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-300 | head -8; tail -1 "$out/pytest_gpu.log"
