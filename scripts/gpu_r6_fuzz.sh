out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 400 python -u scripts/one_launch_fuzz.py --seconds ${2:-240} --out "$out/fuzz.jsonl" > "$out/fuzz.log" 2>&1
rc=$?; echo "fuzz rc=$rc"; tail -5 "$out/fuzz.log"
