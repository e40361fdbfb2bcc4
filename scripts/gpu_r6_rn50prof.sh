# round-6 end tree: ResNet-50 steady-state kernel table with both BatchNorm folds
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/prof_rn50" -o rn50 -- python3 bench.py --model resnet50 --steps 30 --warmup 10 > "$out/bench_prof_rn50.log" 2>&1 || { echo "prof rn50 rc=$?"; exit 1; }
f=$(find "$out/prof_rn50" -name "*kernel_trace.csv" | head -1)
python scripts/kernel_window.py "$f" --window-ms 270 --steps 20 > "$out/kernel_stats_rn50.csv" && head -8 "$out/kernel_stats_rn50.csv" | cut -c1-160
rm -rf "$out/prof_rn50"
