# N > 1 rehearsals on the end-of-round tree (after the uncached-region pool): the
# headline bench with 2 / 4 ranks sharing the one GPU (actor launch and the driver's
# torchrun form), and the ResNet-50 DP step with 2 ranks
out=gpurun_out/$1
mkdir -p "$out"
for n in 2 4; do
  RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus $n --steps 20 --warmup 5 > "$out/share$n.log" 2>&1 || { echo "share$n rc=$?"; tail -5 "$out/share$n.log"; exit 1; }
  echo "share$n $(grep '"metric"' "$out/share$n.log" | cut -c150-420)"
done
RLA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > "$out/torchrun2.log" 2>&1 || { echo "torchrun2 rc=$?"; tail -5 "$out/torchrun2.log"; exit 1; }
echo "torchrun2 $(grep '"metric"' "$out/torchrun2.log" | cut -c150-420)"
RLA_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --model resnet50 --gpus 2 --steps 10 --warmup 5 > "$out/rn50_share2.log" 2>&1 || { echo "rn50 share2 rc=$?"; tail -5 "$out/rn50_share2.log"; exit 1; }
echo "rn50 share2 $(grep '"metric"' "$out/rn50_share2.log" | cut -c100-500)"
