"""Steady-state kernel statistics from a rocprofv3 kernel trace: only kernels that
START inside the last ``--window-ms`` of the trace (the timed steps; warm-up and
MIOpen's solver search come earlier), aggregated by name.

    python scripts/kernel_window.py run_kernel_trace.csv --window-ms 350 --steps 20 > stats.csv
"""
import argparse
import csv
import sys
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--window-ms", type=float, required=True)
ap.add_argument("--steps", type=int, default=1, help="divide totals by this (per-step figures)")
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
name_key = "Kernel_Name" if rows and "Kernel_Name" in rows[0] else "Name"
end = max(int(r["End_Timestamp"]) for r in rows)
lo = end - int(args.window_ms * 1e6)
agg = defaultdict(lambda: [0, 0])
busy = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < lo:
        continue
    a = agg[r[name_key]]
    a[0] += 1
    a[1] += e - s
    busy += e - s
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "PerStepUs", "Percentage"])
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    w.writerow([name, n, t, round(t / args.steps / 1e3, 2), round(100.0 * t / max(busy, 1), 2)])
print(f"# window {args.window_ms} ms, kernel busy {busy / 1e6:.2f} ms "
      f"({busy / 1e3 / args.steps:.1f} us per step over {args.steps} steps)", file=sys.stderr)
