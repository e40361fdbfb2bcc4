# deferred bn2 apply (conv3 applies it in its kernels) + int32 H1pre: tests, then ResNet-50
# A/B (RLA_BN_DEFER=0 / 1, same box), then the MNIST bench
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv1x1_stats.py tests/test_mlp3.py tests/test_fused_validation.py tests/test_dispatch.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"; [ $rc -eq 0 ] || exit 1
for d in 0 1; do
  RLA_BN_DEFER=$d timeout -k 10 300 python -u bench.py --model resnet50 --steps 30 --warmup 10 > "$out/rn50_defer$d.log" 2>&1 || { echo "rn50 defer=$d rc=$?"; exit 1; }
  echo "defer=$d $(tail -1 "$out/rn50_defer$d.log" | cut -c1-200)"
done
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_mnist.log" 2>&1 || { echo "mnist rc=$?"; exit 1; }
tail -1 "$out/bench_mnist.log" | cut -c1-200
