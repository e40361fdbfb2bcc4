"""GPU idle gaps between consecutive kernels of a rocprofv3 kernel trace.

Usage: python scripts/trace_gaps.py <dir with *kernel_trace.csv> [--pattern mlp3]

For every process in the trace: kernels sorted by start; busy = sum of kernel
durations, span = last end - first start, and the gap distribution between
consecutive kernels (the time the GPU queue sat empty: host-bound dispatch,
graph-launch latency, syncs).  Prints one JSON line per process.
"""
import csv
import glob
import json
import os
import statistics
import sys


def main() -> None:
    root = sys.argv[1]
    pat = sys.argv[sys.argv.index("--pattern") + 1] if "--pattern" in sys.argv else None
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    by_pid = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            by_pid.setdefault(r.get("Process_Id", "?"), []).append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for pid, ks in by_pid.items():
        ks.sort()
        if pat:
            # the window from the first to the last matching kernel, all kernels inside it
            idx = [i for i, k in enumerate(ks) if pat in k[2]]
            if not idx:
                continue
            ks = ks[idx[0]: idx[-1] + 1]
        busy = sum(e - s for s, e, _ in ks)
        span = ks[-1][1] - ks[0][0]
        gaps = [max(0, b[0] - a[1]) for a, b in zip(ks, ks[1:])]
        big = sorted(gaps)[-5:]
        names = {}
        for s, e, n in ks:
            short = n.split("(")[0][-60:]
            t = names.setdefault(short, [0, 0])
            t[0] += 1
            t[1] += e - s
        top = sorted(names.items(), key=lambda kv: -kv[1][1])[:8]
        print(json.dumps({
            "pid": pid, "kernels": len(ks), "span_ms": round(span / 1e6, 3), "busy_ms": round(busy / 1e6, 3),
            "busy_frac": round(busy / span, 4) if span else None,
            "gap_median_us": round(statistics.median(gaps) / 1e3, 3) if gaps else None,
            "gap_p99_us": round(sorted(gaps)[int(0.99 * (len(gaps) - 1))] / 1e3, 3) if gaps else None,
            "gap_total_ms": round(sum(gaps) / 1e6, 3), "largest_gaps_us": [round(g / 1e3, 1) for g in big],
            "top_kernels": [{"name": n, "calls": c, "ms": round(t / 1e6, 3)} for n, (c, t) in top],
        }))


if __name__ == "__main__":
    main()
