"""Per-kernel HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python scripts/pmc_bytes.py gpurun_out/r2pmc/pmc_FETCH_SIZE gpurun_out/r2pmc/pmc_WRITE_SIZE

FETCH_SIZE / WRITE_SIZE are the TCC (L2) <-> memory-fabric bytes in KiB per
dispatch.  Prints, per kernel name, the dispatch count and the median KiB per
dispatch summed over all ranks' traces (every rank runs the same sequence).
"""
import collections
import csv
import glob
import os
import statistics
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> pid -> values
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"]][r["Process_Id"]].append(float(r["Counter_Value"]))
    return per


def main():
    out = {}
    for d in sys.argv[1:]:
        name = os.path.basename(d.rstrip("/")).replace("pmc_", "")
        for k, pids in load(d).items():
            if "ccmpi" not in k:
                continue
            n = min(len(v) for v in pids.values())
            med = sum(statistics.median(v) for v in pids.values())  # summed over ranks
            out.setdefault(k, {})[name] = (n, med)
    names = [os.path.basename(d.rstrip("/")).replace("pmc_", "") for d in sys.argv[1:]]
    print("| kernel | dispatches / rank | " + " | ".join(f"{n} MiB (all ranks, median dispatch)" for n in names) + " |")
    print("|---|---:|" + "---:|" * len(names))
    for k, v in sorted(out.items()):
        short = k.split("(")[0].replace("void ccmpi::dev::", "")
        cnt = max(x[0] for x in v.values())
        print(f"| `{short}` | {cnt} | " + " | ".join(f"{v[n][1] / 1024:.1f}" if n in v else "-" for n in names) + " |")


if __name__ == "__main__":
    main()
