# Same-box A/B/C of the MNIST step: base = HEAD's kernel (build/base), g2 = the tree
# (two H1pre copies, 32.32 fixed point), i32 = two copies in 12.20 int32 (build/i32)
out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
dir() { case $1 in base) echo build/base;; i32) echo build/i32;; *) echo .;; esac; }
for rep in 1 2; do
  for v in base g2 i32; do
    (cd $(dir $v) && timeout -k 10 120 python -u $R/scripts/k20_probe.py --graphs 20 --windows 60) > "$out/k20_${v}_$rep.log" 2>&1 || { echo "k20 $v rc=$?"; exit 1; }
    echo "$v $(grep '"graph_steps": 20' "$out/k20_${v}_$rep.log" | cut -c1-200)"
  done
done
for v in base g2 i32; do
  (cd $(dir $v) && timeout -k 10 200 python -u $R/scripts/dp_overhead_probe.py --steps 3000 --worlds 1,8) > "$out/dp_${v}.log" 2>&1 || { echo "dp $v rc=$?"; exit 1; }
  echo "== $v"; grep -v amdgpu.ids "$out/dp_${v}.log" | cut -c1-160
done
for v in base g2 i32; do
  (cd $(dir $v) && timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5) > "$out/bench_${v}.log" 2>&1 || { echo "bench $v rc=$?"; exit 1; }
  echo "$v $(tail -1 "$out/bench_${v}.log" | cut -c1-120)"
done
