# round 6: do non-kernel writes (copies, memsets) reach every XCD's next kernel?
out=gpurun_out/$1
mkdir -p "$out"
for m in 0 1 2 3 4; do
  for b in 4096 12288 65536 614400; do
    timeout -k 10 60 ./build/dma_coherence_probe $m 400 $b >> "$out/dma.jsonl" 2>&1 || { echo "probe $m $b rc=$?"; exit 1; }
  done
done
cat "$out/dma.jsonl"
