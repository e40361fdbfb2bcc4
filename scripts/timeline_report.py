"""Summarise an ``RLA_TIMELINE`` file: per process, each event's offset from the
first event of the run, and the gaps between consecutive events (largest first)."""
import json
import sys
from collections import defaultdict

rows = [json.loads(line) for line in open(sys.argv[1]) if line.strip()]
rows.sort(key=lambda r: r["t"])
t0 = rows[0]["t"]
by_pid = defaultdict(list)
for r in rows:
    by_pid[r["pid"]].append(r)
gaps = []
for pid, rs in by_pid.items():
    print(f"pid {pid}:")
    prev = None
    for r in rs:
        extra = {k: v for k, v in r.items() if k not in ("t", "pid", "event")}
        dt = "" if prev is None else f"(+{(r['t'] - prev['t']) * 1e3:8.1f} ms)"
        print(f"  {(r['t'] - t0):8.3f}s {dt:>14} {r['event']} {extra if extra else ''}")
        if prev is not None:
            gaps.append(((r["t"] - prev["t"]) * 1e3, pid, prev["event"], r["event"]))
        prev = r
print("largest in-process gaps:")
for g in sorted(gaps, reverse=True)[:15]:
    print(f"  {g[0]:9.1f} ms  pid {g[1]}  {g[2]} -> {g[3]}")
if "--merged" in sys.argv:
    print("all processes, in time order:")
    prev = t0
    for r in rows:
        extra = {k: v for k, v in r.items() if k not in ("t", "pid", "event")}
        print(f"  {(r['t'] - t0):8.3f}s (+{(r['t'] - prev) * 1e3:7.1f} ms) pid {r['pid']:>7} {r['event']} "
              f"{extra if extra else ''}")
        prev = r["t"]
