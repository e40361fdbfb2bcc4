#!/bin/bash
# Counter passes (one rocprofv3 --pmc pass per run) of one weight-gradient kernel shape.
#   bash scripts/gpu_wgrad_pmc.sh OUT "<wgrad_one.py args>"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/wpmc}; ARGS=${2:-"--h 56 --cin 64 --cout 64 --k 3"}; mkdir -p "$O"
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$O/p$i" -o run -- python3 scripts/wgrad_one.py $ARGS \
    > "$O/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$O/p$i.log"; exit 1; }
  f=$(find "$O/p$i" -name "*counter_collection.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad" in r.get("Kernel_Name", "") and "reduce" not in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: round(sum(v) / len(v), 1) for k, v in acc.items()})
PY
  rm -rf "$O/p$i"
done
