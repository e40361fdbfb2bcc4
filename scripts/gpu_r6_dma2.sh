out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 150 python -u scripts/dma_stress.py --seconds 90 --out "$out/dma_stress.jsonl" > "$out/dma_stress.log" 2>&1
echo "dma_stress rc=$?"; tail -2 "$out/dma_stress.log"
timeout -k 10 500 python -u -m pytest -s -v --timeout 150 --timeout-method thread tests -m gpu > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -aE "FAILED|FIRST_BAD" "$out/pytest_gpu.log" | cut -c1-300 | head -5; tail -1 "$out/pytest_gpu.log"
