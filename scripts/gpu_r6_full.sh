# round-6 tree: the whole GPU suite (no -x), smoke, the driver-shaped bench, then
# kernel traces of the MNIST bench and the ResNet-50 bench (steady-state tables)
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-400 | head -8; tail -1 "$out/pytest_gpu.log"
[ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_k20.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 "$out/bench_k20.log" | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/prof_mnist" -o mnist -- python3 bench.py --gpus 1 --steps 2000 --warmup 200 > "$out/bench_prof_mnist.log" 2>&1 || { echo "prof mnist rc=$?"; exit 1; }
f=$(find "$out/prof_mnist" -name "*kernel_trace.csv" | head -1)
python scripts/kernel_window.py "$f" --window-ms 15 --steps 1 > "$out/kernel_stats_mnist_window.csv" && head -5 "$out/kernel_stats_mnist_window.csv"
rm -rf "$out/prof_mnist"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/prof_rn50" -o rn50 -- python3 bench.py --model resnet50 --steps 30 --warmup 10 > "$out/bench_prof_rn50.log" 2>&1 || { echo "prof rn50 rc=$?"; exit 1; }
f=$(find "$out/prof_rn50" -name "*kernel_trace.csv" | head -1)
python scripts/kernel_window.py "$f" --window-ms 270 --steps 20 > "$out/kernel_stats_rn50.csv" && head -8 "$out/kernel_stats_rn50.csv" | cut -c1-160
rm -rf "$out/prof_rn50"
