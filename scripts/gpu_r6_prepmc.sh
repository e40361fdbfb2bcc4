# round-6 PRE kernels: device time fused vs unfused, then counter passes (one per run)
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
timeout -k 10 200 python -u scripts/pre_pmc_driver.py --time > "$out/pre_time.log" 2>&1 || { echo "time rc=$?"; tail -20 "$out/pre_time.log"; exit 1; }
cat "$out/pre_time.log" | grep " us "
cd /tmp
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $pass -d "$R/$out/pmc_$tag" -o pmc --output-format csv -- \
    python3 "$R/scripts/pre_pmc_driver.py" > "$R/$out/pmc_$tag.log" 2>&1 || { echo "pmc $tag rc=$?"; tail -20 "$R/$out/pmc_$tag.log"; exit 1; }
  echo "pmc $tag ok"
done
cd "$R"
python scripts/pmc_summary.py $out/pmc_* > "$out/pmc_summary.md" && rm -rf $out/pmc_SQ_WAVES $out/pmc_FETCH_SIZE $out/pmc_WRITE_SIZE
