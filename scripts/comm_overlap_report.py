#!/usr/bin/env python
"""Where the gradient collectives sit against backward, from a rocprofv3 kernel
trace of a data-parallel ResNet-50 run (one ``kernel_trace.csv`` per rank process).

Steps are delimited by the fused SGD kernel.  Per step and rank it reports: the
collective kernels' total device time, the part of it during which a compute
kernel of the same rank was also running (overlapped with backward), and the
EXPOSED time -- from the end of the last compute kernel before the SGD to the SGD's
start, which is what the step pays for communication on the critical path.

Usage: python scripts/comm_overlap_report.py TRACE_DIR [--last 10] [--timeline OUT_PREFIX]
(--timeline: per rank, the last step's kernels as CSV -- offset from the step start,
duration, comm or compute -- small enough to commit next to the summary)
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics

COMM = ("twoshot_allreduce", "oneshot_allreduce", "ncclDevKernel", "ncclKernel", "rccl", "pack_kernel")


def _is_comm(name: str) -> bool:
    return any(k in name for k in COMM)


def _load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((s, e, name))
    rows.sort()
    return rows


def _overlap(a0, a1, iv):
    """Length of [a0, a1) covered by the union of intervals iv (sorted, merged)."""
    tot = 0
    for s, e in iv:
        if e <= a0:
            continue
        if s >= a1:
            break
        tot += min(a1, e) - max(a0, s)
    return tot


def _merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def timeline(path, out):
    rows = _load(path)
    sgd = [i for i, (_, _, n) in enumerate(rows) if "sgd_kernel" in n]
    if len(sgd) < 2:
        return
    a, b = sgd[-2], sgd[-1]
    t0 = rows[a][1]
    with open(out, "w") as f:
        f.write("start_us,dur_us,kind,kernel\n")
        for s, e, n in rows[a + 1:b + 1]:
            short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            short = short.replace(",", ";")[:120]
            f.write(f"{(s - t0) / 1e3:.1f},{(e - s) / 1e3:.1f},{'comm' if _is_comm(n) else 'compute'},{short}\n")


def report(path, last):
    rows = _load(path)
    sgd = [i for i, (_, _, n) in enumerate(rows) if "sgd_kernel" in n]
    steps = []
    for a, b in zip(sgd, sgd[1:]):
        seg = rows[a + 1:b + 1]  # this step's kernels, ending with its SGD
        t0, t_sgd = seg[0][0], seg[-1][0]
        comm = [(s, e) for s, e, n in seg if _is_comm(n)]
        comp = [(s, e) for s, e, n in seg[:-1] if not _is_comm(n)]
        comp_m = _merge(comp)
        comm_t = sum(e - s for s, e in comm)
        ov = sum(_overlap(s, e, comp_m) for s, e in comm)
        last_comp = max((e for s, e in comp), default=t0)
        steps.append({"step_us": (seg[-1][1] - rows[a][1]) / 1e3, "comm_kernels": len(comm),
                      "comm_us": comm_t / 1e3, "comm_overlapped_us": ov / 1e3,
                      "exposed_us": max(0, t_sgd - last_comp) / 1e3,
                      "first_comm_at_pct": (100.0 * (min(s for s, _ in comm) - t0) / max(1, t_sgd - t0)) if comm else None})
    steps = steps[-last:]
    if not steps:
        return None
    med = {k: round(statistics.median([s[k] for s in steps if s[k] is not None]), 2)
           for k in steps[0] if steps[0][k] is not None}
    return {"trace": os.path.relpath(path), "steps": len(steps), "median": med}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--timeline", default=None)
    args = ap.parse_args(argv)
    paths = sorted(glob.glob(os.path.join(args.trace_dir, "**", "*kernel_trace.csv"), recursive=True))
    for i, p in enumerate(paths):
        if args.timeline:
            timeline(p, f"{args.timeline}_{i}.csv")
    for p in paths:
        r = report(p, args.last)
        if r is not None:
            print(json.dumps(r))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
