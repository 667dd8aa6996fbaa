"""Markdown tables from benchmarks/coll_sweep.py JSONL output.

    python scripts/coll_table.py profiles/r2_coll/all_p8.jsonl [--metric hbm_frac|us|busbw_GBps]
"""
import argparse
import collections
import json


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--metric", default="both", help="us | hbm_frac | busbw_GBps | algbw_GBps | both (us / hbm_frac)")
    a = ap.parse_args()
    for f in a.files:
        rows = collections.OrderedDict()
        sizes = set()
        ranks = None
        for line in open(f):
            r = json.loads(line)
            ranks = r["ranks"]
            sizes.add(r["size"])
            key = (r["op"], r["algo"])
            if "error" in r:
                rows.setdefault(key, {})[r["size"]] = "err"
            elif a.metric == "both":
                rows.setdefault(key, {})[r["size"]] = f"{r['us']:.0f} / {r['hbm_frac']:.2f}"
            else:
                rows.setdefault(key, {})[r["size"]] = f"{r[a.metric]}"
        sizes = sorted(sizes)
        label = "us / HBM fraction" if a.metric == "both" else a.metric
        print(f"#### {f.split('/')[-1]}: {ranks} ranks, {label}\n")
        hdr = ["op", "algo"] + [(f"{s >> 20} MiB" if s >= 1 << 20 else f"{s >> 10} KiB") for s in sizes]
        print("| " + " | ".join(hdr) + " |")
        print("|" + "---|" * 2 + "---:|" * len(sizes))
        for (op, algo), v in rows.items():
            print(f"| {op} | {algo} | " + " | ".join(v.get(s, "-") for s in sizes) + " |")
        print()


if __name__ == "__main__":
    main()
