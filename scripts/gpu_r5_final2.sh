# round-5 final numbers after the fork revert + the restored MNIST head change
set -o pipefail
O=gpurun_out/r5_final2; mkdir -p $O
bash scripts/gpu_stage.sh $O rn50graph rn50prof || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_mlp3.py > $O/pytest_mlp3.log 2>&1 || { tail -20 $O/pytest_mlp3.log; exit 1; }
tail -1 $O/pytest_mlp3.log
for i in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20_$i.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' $O/bench_k20_$i.log; done
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' $O/bench_default.log
bash scripts/gpu_stage.sh $O rn50trainer
