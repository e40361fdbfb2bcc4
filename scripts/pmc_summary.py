"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one or more passes).

  python scripts/pmc_summary.py DIR [DIR ...] > summary.md
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("rla::", "")
    return name.split("(")[0][:90]


def main(dirs):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    k = short(r.get("Kernel_Name", ""))
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    counters = sorted({c for k in vals for c in vals[k]})
    print("| kernel | " + " | ".join(counters) + " | VALU / MFMA-busy cycle | LDS conflict / LDS-active |")
    print("|---|" + "---|" * (len(counters) + 2))
    for k in sorted(vals):
        avg = {c: (sum(v) / len(v) if v else 0.0) for c, v in vals[k].items()}
        row = [f"{avg.get(c, 0):.4g}" for c in counters]
        mfma = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        valu = avg.get("SQ_INSTS_VALU", 0)
        lds_a, lds_c = avg.get("SQ_LDS_IDX_ACTIVE", 0), avg.get("SQ_LDS_BANK_CONFLICT", 0)
        ratio = f"{valu / mfma:.3f}" if mfma else "-"
        conf = f"{lds_c / lds_a:.3f}" if lds_a else "-"
        print(f"| {k} | " + " | ".join(row) + f" | {ratio} | {conf} |")


if __name__ == "__main__":
    main(sys.argv[1:])
