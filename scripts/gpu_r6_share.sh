# N > 1 rehearsal of the headline bench: 2 and 4 ranks sharing the one GPU
out=gpurun_out/$1
mkdir -p "$out"
for n in 2 4; do
  RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus $n --steps 20 --warmup 5 > "$out/share$n.log" 2>&1 || { echo "share$n rc=$?"; tail -5 "$out/share$n.log"; exit 1; }
  echo "share$n $(grep '"metric"' "$out/share$n.log" | cut -c150-420)"
done
