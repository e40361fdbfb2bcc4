# BASELINE configs 3 and 4 on the end-of-round tree (ranks / trials sharing the one GPU):
# Horovod route at 2 ranks, and the Tune sweep (4 trials x 2 workers, recycled workers)
out=gpurun_out/$1
mkdir -p "$out"
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --accelerator horovod --steps 20 --warmup 5 > "$out/horovod2.log" 2>&1 || { echo "horovod2 rc=$?"; tail -5 "$out/horovod2.log"; exit 1; }
echo "horovod2 $(grep '"metric"' "$out/horovod2.log" | cut -c150-420)"
timeout -k 10 400 python -u scripts/bench_tune.py --workers 2 --share-gpu 8 --trials 4 --epochs 2 > "$out/tune_cfg4.log" 2>&1 || { echo "tune rc=$?"; tail -5 "$out/tune_cfg4.log"; exit 1; }
tail -2 "$out/tune_cfg4.log" | cut -c1-400
