# bn1 -> conv2 deferral: kernel and block tests, then ResNet-50 A/B on one box
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv3x3.py tests/test_conv1x1_stats.py tests/test_conv_wgrad.py tests/test_bn.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"; [ $rc -eq 0 ] || exit 1
for d in 0 1; do
  RLA_BN_DEFER=$d timeout -k 10 300 python -u bench.py --model resnet50 --steps 30 --warmup 10 > "$out/rn50_defer$d.log" 2>&1 || { echo "rn50 defer=$d rc=$?"; exit 1; }
  echo "defer=$d $(grep '"metric"' "$out/rn50_defer$d.log" | cut -c1-160)"
done
python - "$out/rn50_defer1.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print({k: v for k, v in d.get("conv1x1_backends", {}).items() if "pre" in k})
PY
