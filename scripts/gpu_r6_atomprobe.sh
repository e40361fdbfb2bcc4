out=gpurun_out/$1
mkdir -p "$out"
R=$(pwd)
for rep in 1 2; do
for v in tree noatom; do
  if [ $v = tree ]; then d=.; else d=build/probe_noatom; fi
  (cd $d && timeout -k 10 120 python -u $R/scripts/k20_probe.py --graphs 20 --windows 40) > "$out/k20_${v}_$rep.log" 2>&1 || { echo "k20 $v rc=$?"; exit 1; }
  echo "$v $(grep '"graph_steps": 20' $out/k20_${v}_$rep.log | cut -c1-160)"
  (cd $d && timeout -k 10 120 python -u $R/scripts/dp_phase_probe.py plain) > "$out/ph_${v}_$rep.log" 2>&1 || { echo "ph $v rc=$?"; exit 1; }
  echo "$v $(grep plain $out/ph_${v}_$rep.log | cut -c1-500)"
done
done
