# framework-path numbers on the round-6 tree: Trainer.fit MNIST and ResNet-50 (with the
# resident validation split and a checkpoint every epoch), plus the default MNIST bench
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 300 python -u bench.py --via trainer > "$out/mnist_trainer.log" 2>&1 || { echo "mnist trainer rc=$?"; exit 1; }
echo "mnist trainer $(grep '"metric"' "$out/mnist_trainer.log" | cut -c1-220)"
timeout -k 10 500 python -u bench.py --via trainer --model resnet50 > "$out/rn50_trainer.log" 2>&1 || { echo "rn50 trainer rc=$?"; exit 1; }
python - "$out/rn50_trainer.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        keep = ("value", "value_without_validation", "ms_per_step", "val_loss", "val_accuracy", "train_steps_per_epoch",
                "checkpointing", "val_batches_per_epoch", "final_train_loss")
        print("rn50 trainer", {k: d.get(k, d.get("config", {}).get(k)) for k in keep})
PY
timeout -k 10 300 python -u bench.py --model resnet50 --steps 30 --warmup 10 > "$out/rn50_engine.log" 2>&1 || { echo "rn50 engine rc=$?"; exit 1; }
echo "rn50 engine $(grep '"metric"' "$out/rn50_engine.log" | cut -c60-140)"
timeout -k 10 300 python -u bench.py > "$out/mnist_default.log" 2>&1 || { echo "mnist default rc=$?"; exit 1; }
echo "mnist default $(grep '"metric"' "$out/mnist_default.log" | cut -c100-260)"
