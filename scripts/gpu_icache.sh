#!/bin/bash
# Instruction-cache counters of the one-launch MNIST step: plain vs loopback DP variants
# (one rocprofv3 --pmc pass per run, each under its own limit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/icache}; mkdir -p "$O"
for v in "none 1" "packed 1" "packed 8" "owner 8"; do
  set -- $v
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES \
    --output-format csv -d "$O/pmc_$1_$2" -o run -- python3 scripts/dp_variant_run.py --proto $1 --world $2 \
    > "$O/pmc_$1_$2.log" 2>&1 || { echo "pmc $1 $2 failed"; tail -20 "$O/pmc_$1_$2.log"; exit 1; }
  f=$(find "$O/pmc_$1_$2" -name "*counter_collection.csv" | head -1)
  python - "$f" "$1 $2" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "one_kernel" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(v) / len(v), 1) for k, v in acc.items()}, "dispatches", len(acc.get("SQ_WAVES", [])))
PY
  rm -rf "$O/pmc_$1_$2"
done
