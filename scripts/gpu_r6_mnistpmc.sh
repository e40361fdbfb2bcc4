# counter passes over the round-6 one-launch MNIST step (bench.py, 1 GPU), one pass per run
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
cd /tmp
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass -d "$R/$out/pmc_$tag" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --gpus 1 --steps 200 --warmup 20 > "$R/$out/pmc_$tag.log" 2>&1 || { echo "pmc $tag rc=$?"; tail -20 "$R/$out/pmc_$tag.log"; exit 1; }
  echo "pmc $tag ok"
done
cd "$R"
python scripts/pmc_summary.py $out/pmc_* > "$out/pmc_summary.md" && grep mlp3 "$out/pmc_summary.md" | cut -c1-300
rm -rf $out/pmc_SQ_WAVES $out/pmc_SQ_WAIT_INST_ANY $out/pmc_FETCH_SIZE $out/pmc_WRITE_SIZE
