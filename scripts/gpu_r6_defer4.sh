# packed BN-ReLU transform: kernel and block tests, then ResNet-50 on one box with
# no deferral / bn2 only (bn1 materialised) / both (timed per shape)
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv3x3.py tests/test_conv1x1_stats.py tests/test_conv_wgrad.py tests/test_bn.py -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 "$out/tests.log"; [ $rc -eq 0 ] || exit 1
for v in off bn2 both; do
  case $v in off) e="RLA_BN_DEFER=0";; bn2) e="RLA_CONV3X3_PRE=apply";; both) e="RLA_BN_DEFER=1";; esac
  env $e timeout -k 10 300 python -u bench.py --model resnet50 --steps 30 --warmup 10 > "$out/rn50_$v.log" 2>&1 || { echo "rn50 $v rc=$?"; exit 1; }
  echo "$v $(grep '"metric"' "$out/rn50_$v.log" | cut -c60-130)"
done
python - "$out/rn50_both.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print({k: v for k, v in d.get("conv1x1_backends", {}).items() if "pre" in k or k.startswith("wgrad_kxk 4014")})
PY
