#!/bin/bash
# Parameterised GPU stages (one gpurun call runs several, chained; each GPU step under
# its own limit; the first failing step ends the call).
#   bash scripts/gpu_stage.sh OUT STAGE [STAGE ...]
# stages: suite (full GPU pytest + smoke + default bench), dp (exchange protocols:
# loopback / 2-rank tests + per-N cost probe + phase stamps), dpphase, tune (sweep
# trials/hour cold + warm), trainer (Trainer.fit bench + epoch-boundary timeline),
# recycle (worker reuse tests), prof (rocprofv3 kernel stats of the default bench),
# pmc (counter passes of the default step, one pass per run), bench20 (driver-shaped
# bench), share2 (N = 2 rehearsals with both ranks on the one GPU), corners (Tune
# search-space corners), selftest (native comm self-test, plain + host ASan/UBSan),
# wgrad (conv weight-gradient kernel tests + probe), rn50b (native ResNet-50 bench),
# c1stats (1x1 conv + BN statistics kernel),
# rn50 (ResNet-50 bench, native + stock torch; --deterministic-conv
# is not run: MIOpen's atomic-free solvers compile for > 3 min without output), rn50prof (its kernel stats)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=${1:-gpurun_out/stage}; shift; mkdir -p "$O"
run() {  # name limit cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] FAILED rc=$rc"; tail -40 "$O/$n.log"; exit $rc; fi
  echo "[$n] ok"; grep -h '^{' "$O/$n.log" | cut -c1-600 || true
}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
for st in "$@"; do
  case $st in
    suite)
      run pytest_gpu 1200 $PYT tests -m gpu
      tail -3 "$O/pytest_gpu.log"
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      run bench_default 300 python bench.py ;;
    k20)  # the driver's bench window
      run bench_k20 300 python bench.py --steps 20 --warmup 5 ;;
    dp)
      RLA_FIDELITY_LOG="$R/$O/fidelity.jsonl" run pytest_dp 600 $PYT tests/test_mlp3.py tests/test_comm.py -k "loopback or fused_dp or fp32"
      run dp_probe 300 python -u scripts/dp_overhead_probe.py
      run dp_phases 300 python -u scripts/dp_phase_probe.py ;;
    dpphase)
      run dp_phases 300 python -u scripts/dp_phase_probe.py ;;
    recycle)
      run pytest_recycle 300 $PYT tests/test_ddp_gpu.py tests/test_runtime.py -k "recycl" ;;
    c3pmc)  # counter passes over the 3x3 MFMA convolution, one pass per run
      cd /tmp
      for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
        tag=$(echo $pass | cut -d' ' -f1)
        timeout -s KILL 90 rocprofv3 --pmc $pass -d "$R/$O/c3pmc_$tag" -o pmc --output-format csv -- \
          python "$R/scripts/conv3x3_pmc.py" > "$R/$O/c3pmc_$tag.log" 2>&1 || { echo "[c3pmc $tag] FAILED"; tail -20 "$R/$O/c3pmc_$tag.log"; exit 1; }
        echo "[c3pmc $tag] ok"
      done
      cd "$R" ;;
    tuneaudit)  # config 4 (2 workers sharing the GPU, recycled) with per-fit worker diagnostics audited
      run tune_audit 240 python -u scripts/bench_tune.py --workers 2 --share-gpu 8 --trials 8 --epochs 2 --diag-dir "$R/$O/tune_diag" ;;
    tune)
      run tune_cold 300 python scripts/bench_tune.py --trials 4
      run tune_cold16 300 python scripts/bench_tune.py --trials 16
      run tune_warm 300 python scripts/bench_tune.py --trials 8 --warm 8 ;;
    trainerprof)  # host profile of the worker's fit (cProfile, rank 0)
      RLA_PROFILE_EPOCHS="$R/$O/trainer_epochs_prof" run trainer_prof 300 python bench.py --via trainer --trainer-epochs 6 ;;
    wgrad)  # MFMA conv weight-gradient kernel: numerics + per-shape timing vs MIOpen / hipBLASLt
      run pytest_wgrad 300 $PYT tests/test_conv_wgrad.py tests/test_bn.py
      run wgrad_probe 300 python -u scripts/wgrad_probe.py ;;
    wsplit)  # weight-gradient split-count sweep (planner's S vs fixed S per shape)
      run wgrad_split 600 python -u scripts/wgrad_split_sweep.py ;;
    rn50b)  # native ResNet-50 bench: eager and whole-step hipGraph
      run rn50_base 600 python bench.py --model resnet50 --steps 30 --warmup 10
      run rn50_graph 600 python bench.py --model resnet50 --steps 30 --warmup 10 --resnet-graph 1 ;;
    rn50graph)
      run rn50_graph 600 python bench.py --model resnet50 --steps 30 --warmup 10 --resnet-graph 1 ;;
    rn50host)  # host cProfile of the eager native ResNet-50 step
      run rn50_host 300 python -u scripts/rn50_host_prof.py ;;
    rn50ops)
      run rn50_ops 300 python -u scripts/rn50_op_profile.py ;;
    conv1x1)
      run conv1x1 300 python -u scripts/conv1x1_probe.py ;;
    c1stats)  # 1x1 forward with BN statistics in the epilogue: tests + per-shape timing
      run pytest_c1stats 300 $PYT tests/test_conv1x1_stats.py tests/test_bn.py -m gpu
      run c1stats_probe 300 python -u scripts/conv1x1_stats_probe.py ;;
    tunetl)  # cold sweep with the cross-process start-up timeline
      RLA_TIMELINE="$R/$O/tune_timeline.jsonl" run tune_tl 300 python scripts/bench_tune.py --trials 6
      python scripts/timeline_report.py "$O/tune_timeline.jsonl" --merged > "$O/tune_timeline.txt" 2>&1 || true ;;
    trainertests)  # Trainer / checkpoint GPU tests
      run pytest_trainer 600 $PYT tests/test_checkpoint_writer.py tests/test_dispatch.py tests/test_fused_validation.py tests/test_trainer.py -m gpu ;;
    trainer)
      RLA_TIMELINE="$R/$O/trainer_timeline.jsonl" run trainer 300 python bench.py --via trainer --trainer-epochs 6
      python scripts/timeline_report.py "$O/trainer_timeline.jsonl" > "$O/trainer_timeline.txt" 2>&1 || true ;;
    prof)
      run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py"
      find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_default.csv" \;
      rm -rf "$O/prof" ;;  # raw traces exceed gpurun's 64 MiB copy-back
    bench20)
      run bench_k20 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    rn50)
      run pytest_bn 300 $PYT tests/test_bn.py
      RB="python bench.py --model resnet50 --steps 30 --warmup 10"
      run rn50_base 600 $RB
      run rn50_torch 600 $RB --impl torch ;;
    rn50prof)
      run rn50_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/rn50prof" -o run -- \
        python3 "$R/bench.py" --model resnet50 --steps 20 --warmup 10
      find "$O/rn50prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_rn50_all.csv" \;
      # steady state: the last 20 steps (MIOpen's find runs during warm-up on a fresh box)
      MS=$(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['ms_per_step'])" "$O/rn50_prof.log")
      python scripts/kernel_window.py "$(find "$O/rn50prof" -name '*kernel_trace.csv' | head -1)" \
        --window-ms "$(python -c "print($MS * 20)")" --steps 20 > "$O/kernel_stats_rn50.csv" 2> "$O/kernel_window.txt"
      rm -rf "$O/rn50prof" ;;
    pmc)
      B="python bench.py --steps 300 --warmup 30 --graph-steps 0"
      for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
                  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
        n=$(echo $pass | cut -d' ' -f1)
        timeout -s KILL 60 rocprofv3 --pmc $pass --output-format csv -d "$O/pmc_$n" -o run -- $B > "$O/pmc_$n.log" 2>&1 \
          || { echo "pmc pass $n failed"; tail -20 "$O/pmc_$n.log"; exit 1; }
      done
      find "$O" -name "*counter_collection.csv" ;;
    pmc5)  # counter passes over the round-5 convolution kernels only (scripts/kernel_pmc_driver.py)
      cd /tmp
      for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
                  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
        n=$(echo $pass | cut -d' ' -f1)
        timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$R/$O/pmc5_$n" -o run -- \
          python3 "$R/scripts/kernel_pmc_driver.py" > "$R/$O/pmc5_$n.log" 2>&1 \
          || { echo "pmc pass $n failed"; tail -20 "$R/$O/pmc5_$n.log"; exit 1; }
      done
      cd "$R"
      python scripts/pmc_summary.py $O/pmc5_* > "$O/pmc5_summary.md" && cat "$O/pmc5_summary.md" ;;
    share2)
      RLA_BENCH_SHARE_GPU=1 run share2_ray 300 python bench.py --gpus 2 --steps 500 --warmup 50
      RLA_BENCH_SHARE_GPU=1 run share2_hvd 300 python bench.py --gpus 2 --steps 500 --warmup 50 --accelerator horovod
      RLA_BENCH_SHARE_GPU=1 run share2_torchrun 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 500 --warmup 50 ;;
    corners)
      for c in "128 256 128" "128 256 32" "64 128 64" "32 256 32"; do
        set -- $c
        run corner_$1_$2_b$3 300 python bench.py --layer-1 $1 --layer-2 $2 --batch-size $3
      done ;;
    selftest)
      run selftest_w2 120 ./build/comm_selftest 2
      run selftest_w4 180 ./build/comm_selftest 4
      ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1:protect_shadow_gap=0 \
      LSAN_OPTIONS=suppressions=$R/scripts/sanitizers/lsan.supp:print_suppressions=0 \
      UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 run selftest_asan_w2 300 ./build/comm_selftest_asan 2 ;;
    graphstep)  # Trainer-level graph-captured autograd step: tests + config 5 through Trainer.fit
      run pytest_graph 600 $PYT tests/test_graph_step.py
      run rn50_trainer 900 python -u bench.py --via trainer --model resnet50 --steps 20 --trainer-epochs 4
      run rn50_engine 600 python bench.py --model resnet50 --steps 30 --warmup 10 ;;
    r5tests)  # round-5 GPU tests: comm matrix worlds 1-8, exact buffer broadcast, fused-dgrad guard, graph step
      run pytest_r5 900 $PYT tests/test_comm.py tests/test_conv1x1_stats.py tests/test_graph_step.py \
        -m gpu -k "matrix or bcast_exact or guard or graph or captured" ;;
    comm5)  # config-5 communication on one GPU (proxies): bucket timings, wire trajectory, overlap trace
      run comm_buckets2 300 python -u scripts/comm_quantify.py buckets --world 2
      run comm_buckets8 600 python -u scripts/comm_quantify.py buckets --world 8 --reps 10
      run comm_traj 900 python -u scripts/comm_quantify.py trajectory --steps 300 ;;
    comm5trace)  # kernel trace of the captured 2-rank share-GPU ResNet step: one rocprofv3 per rank process
      cd /tmp
      for r in 0 1; do
        RLA_BENCH_SHARE_GPU=1 RANK=$r WORLD_SIZE=2 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 \
          timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/rn50s2trace/r$r" -o run -- \
          python3 "$R/bench.py" --model resnet50 --gpus 2 --steps 20 --warmup 5 > "$R/$O/rn50s2trace_r$r.log" 2>&1 &
      done
      wait -n || { echo "[comm5trace] a rank failed"; tail -30 "$R/$O/rn50s2trace_r0.log"; exit 1; }
      wait -n || { echo "[comm5trace] a rank failed"; tail -30 "$R/$O/rn50s2trace_r1.log"; exit 1; }
      cd "$R"
      python scripts/comm_overlap_report.py "$O/rn50s2trace" --last 10 > "$O/comm_overlap.jsonl" && cat "$O/comm_overlap.jsonl"
      find "$O/rn50s2trace" -name "*kernel_trace.csv" -size +20M -delete ;;
    c3ab)  # 3x3 MFMA convolution: numerics + fixed-shape vs run-time-shape instances, per shape vs MIOpen
      run pytest_c3 300 $PYT tests/test_conv3x3.py
      run c3probe_fixed 300 python -u scripts/conv3x3_probe.py
      RLA_CONV3X3_GENERIC=1 run c3probe_generic 300 python -u scripts/conv3x3_probe.py ;;
    c3pipe)  # 3x3 MFMA convolution after a schedule change: numerics + per-shape time vs MIOpen
      run pytest_c3 300 $PYT tests/test_conv3x3.py
      run c3probe 300 python -u scripts/conv3x3_probe.py ;;
    wtests)  # weight-gradient + 3x3 kernels numerics
      run pytest_w 300 $PYT tests/test_conv_wgrad.py tests/test_conv3x3.py ;;
    stem)  # ResNet stem kernel: numerics + device time vs MIOpen (+ BN statistics)
      run pytest_stem 300 $PYT tests/test_conv3x3.py -k "stem or maxpool"
      run stem_probe 300 python -u scripts/stem_probe.py ;;
    mnist5)  # one-launch MNIST step after a kernel change: numerics, headline bench, phase stamps, DP cost
      run pytest_mlp3 600 $PYT tests/test_mlp3.py
      run bench_default 300 python bench.py
      run bench_k20 300 python bench.py --gpus 1 --steps 20 --warmup 5
      run dp_phases 300 python -u scripts/dp_phase_probe.py
      run dp_probe 300 python -u scripts/dp_overhead_probe.py ;;
    rn50trainer)
      run rn50_trainer 900 python -u bench.py --via trainer --model resnet50 --steps 20 --trainer-epochs 4 ;;
    rn50share2)  # config 5 through Trainer.fit, 2 ranks sharing the GPU (graph-captured DP step)
      RLA_BENCH_SHARE_GPU=1 run rn50_share2_trainer 900 python -u bench.py --via trainer --model resnet50 --gpus 2 \
        --steps 10 --trainer-epochs 3 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
