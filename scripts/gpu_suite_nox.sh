# the whole GPU suite WITHOUT -x (every failure listed), then smoke
mkdir -p "$1"
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > "$1/pytest_gpu.log" 2>&1
echo "pytest rc=$?"; grep -E "FAILED|ERROR" "$1/pytest_gpu.log" | head -20; tail -2 "$1/pytest_gpu.log"
