# round-6 final tree: the GPU suite as the driver runs it, smoke, the driver-shaped
# bench, and a steady-state MNIST kernel table
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-300 | head -5; tail -1 "$out/pytest_gpu.log"
[ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_k20.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 "$out/bench_k20.log" | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof" -o mnist -- python3 bench.py --gpus 1 --steps 2000 --warmup 200 > "$out/bench_prof.log" 2>&1 || { echo "prof rc=$?"; exit 1; }
f=$(find "$out/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$out/kernel_stats_mnist.csv" && head -4 "$out/kernel_stats_mnist.csv" | cut -c1-200
rm -rf "$out/prof"
