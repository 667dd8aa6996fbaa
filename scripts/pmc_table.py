"""Median per-dispatch PMC counters of the dominant kernel in each rocprofv3 --pmc run.

    python scripts/pmc_table.py gpurun_out/gemm_pmc/pmc_m5_P1 gpurun_out/gemm_pmc/pmc_m5_P2 ...

Each argument is one --pmc output directory.  For every directory, the kernel with the
most dispatches x largest counters (GEMM kernels: names with 'gemm' or 'Cijk' first) is
picked and its counters printed as `counter: median value per dispatch`; rows of the
same label (directory name minus its _P<n> suffix) are merged into one table line.
"""
import collections
import csv
import glob
import os
import re
import statistics
import sys


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            # sum over instances of one dispatch, then median over dispatches
            vals[r["Kernel_Name"]][r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id", "0"))] += \
                float(r["Counter_Value"])
    return vals


def pick(vals):
    names = list(vals)
    pref = [n for n in names if re.search(r"gemm|Cijk", n)]
    pool = pref or names
    return max(pool, key=lambda n: max(len(c) for c in vals[n].values()))


def main():
    rows = collections.OrderedDict()
    for d in sys.argv[1:]:
        vals = load(d)
        if not vals:
            continue
        k = pick(vals)
        label = re.sub(r"_P\d+$", "", os.path.basename(d.rstrip("/")))
        row = rows.setdefault(label, {"kernel": k})
        for c, per in vals[k].items():
            row[c] = statistics.median(per.values())
    cols = sorted({c for r in rows.values() for c in r if c != "kernel"})
    print("| run | kernel | " + " | ".join(cols) + " |")
    print("|---|---|" + "---:|" * len(cols))
    for label, r in rows.items():
        name = r["kernel"][:60]
        print(f"| {label} | `{name}` | " + " | ".join(f"{r.get(c, float('nan')):.4g}" for c in cols) + " |")


if __name__ == "__main__":
    main()
