out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 120 python -u scripts/dp_phase_probe.py > "$out/phases.log" 2>&1; echo "phases rc=$?"; grep -v amdgpu.ids "$out/phases.log"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o mnist -- python3 bench.py --gpus 1 --steps 2000 --warmup 200 > "$out/bench_prof.log" 2>&1; echo "prof rc=$?"
find "$out/prof" -name "*kernel_stats.csv" | head -3
