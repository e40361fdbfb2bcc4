# every GPU test file up to and including tests/test_mlp3.py, one process (the MNIST
# fidelity failure only shows in that session); the failing test prints FIRST_BAD
mkdir -p "$1"
F=$(ls tests/test_*.py | awk '$0 <= "tests/test_mlp3.py"')
timeout -k 10 900 python -u -m pytest -v -rA --timeout 120 --timeout-method thread -m gpu $F > "$1/pytest.log" 2>&1
echo "pytest rc=$?"; grep -a "FIRST_BAD" "$1/pytest.log" | cut -c1-6000; tail -2 "$1/pytest.log"
