# round-6 end-of-round record of the committed tree: the GPU suite as the driver runs it,
# smoke, the driver-shaped MNIST bench, and the config-5 pair (engine, Trainer.fit)
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-300 | head -5; tail -1 "$out/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_k20.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 "$out/bench_k20.log" | cut -c1-200
timeout -k 10 300 python -u bench.py --model resnet50 --steps 30 --warmup 10 > "$out/rn50_graph.log" 2>&1 || { echo "rn50 rc=$?"; exit 1; }
grep '"metric"' "$out/rn50_graph.log" | cut -c1-200
timeout -k 10 400 python -u bench.py --via trainer --model resnet50 > "$out/rn50_trainer.log" 2>&1 || { echo "rn50 trainer rc=$?"; exit 1; }
grep '"metric"' "$out/rn50_trainer.log" | cut -c1-260
