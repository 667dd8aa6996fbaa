"""Median kernel duration per (kernel, grid) over every rank's rocprofv3 kernel trace.

    python scripts/kernel_durations.py gpurun_out/r2lld/prof8 [--match k_allreduce]
"""
import argparse
import collections
import csv
import glob
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--match", default="ccmpi")
a = ap.parse_args()
d = collections.defaultdict(list)
for f in glob.glob(os.path.join(a.dir, "*kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        if a.match in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("(")[0].replace("void ccmpi::dev::", "")
            d[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("| kernel | grid threads | dispatches | median us | p10 us |")
print("|---|---:|---:|---:|---:|")
for (k, g), v in sorted(d.items()):
    v.sort()
    print(f"| `{k}` | {g} | {len(v)} | {statistics.median(v):.2f} | {v[len(v) // 10]:.2f} |")
