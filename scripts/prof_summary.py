"""Summarise rocprofv3 kernel_stats.csv files into a markdown table.

    python scripts/prof_summary.py gpurun_out/prof/harness_tp2 > profiles/x/summary.md
"""
import csv
import glob
import os
import sys


def main(d: str, top: int = 15) -> None:
    files = sorted(glob.glob(os.path.join(d, "*kernel_stats.csv")))
    for f in files:
        rows = list(csv.DictReader(open(f)))
        print(f"### {os.path.basename(f)}\n")
        print("| kernel | calls | total ms | avg us | min us | max us | % |")
        print("|---|---:|---:|---:|---:|---:|---:|")
        for r in rows[:top]:
            name = r["Name"].replace("|", "/")
            if len(name) > 95:
                name = name[:92] + "..."
            print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                  f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                  f"{float(r['Percentage']):.2f} |")
        print()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
