"""Markdown tables from rocprofv3 ``--stats`` CSVs (``*_kernel_stats.csv``): one table per file,
kernels by total time.  Usage: python tools/kernel_stats_md.py <dir> [top] > kernels.md"""
import csv
import glob
import os
import sys


def table(path: str, top: int) -> str:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: -float(r["TotalDurationNs"]))
    out = [f"### {os.path.basename(path)}", "", "| kernel | calls | total ms | avg us | min us | max us | % |",
           "|---|---:|---:|---:|---:|---:|---:|"]
    for r in rows[:top]:
        name = r["Name"] if len(r["Name"]) <= 90 else r["Name"][:90] + "..."
        out.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                   f"{float(r['Percentage']):.2f} |")
    return "\n".join(out) + "\n"


def main() -> None:
    root = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    for p in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
        print(table(p, top))


if __name__ == "__main__":
    main()
