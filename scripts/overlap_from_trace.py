"""Comm/compute overlap from a rocprofv3 kernel trace.

    python scripts/overlap_from_trace.py gpurun_out/ov/prof [--comm k_allreduce,k_move] [--compute gemm]

For every rank's ``*_kernel_trace.csv``: the union of the communication
kernels' busy intervals (C), of the compute kernels' intervals (G), and of
their intersection (C and G running at the same time on that rank's queues).
``overlap_of_comm`` = |C and G| / |C|: the share of communication-kernel time
during which a compute kernel of the same rank was also running.  Prints a
markdown table and the concurrent intervals' first examples.
"""
import argparse
import csv
import glob
import os


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def total(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--comm", default="k_allreduce,k_move,k_reduce_scatter,k_lastaxis")
    ap.add_argument("--compute", default="gemm")
    ap.add_argument("--skip-first-ms", type=float, default=0.0, help="ignore the trace's first ms (setup)")
    a = ap.parse_args()
    comm_keys = a.comm.split(",")
    comp_keys = a.compute.split(",")
    print("| trace | comm kernels | comm busy ms | compute busy ms | concurrent ms | overlap_of_comm |")
    print("|---|---:|---:|---:|---:|---:|")
    for f in sorted(glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))):
        rows = list(csv.DictReader(open(f)))
        t0 = min(int(r["Start_Timestamp"]) for r in rows) + int(a.skip_first_ms * 1e6)
        C, G = [], []
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s < t0:
                continue
            n = r["Kernel_Name"]
            if any(k in n for k in comm_keys):
                C.append([s, e])
            elif any(k in n for k in comp_keys):
                G.append([s, e])
        cu, gu = union(C), union(G)
        both = intersect(cu, gu)
        tc = total(cu)
        frac = total(both) / tc if tc else 0.0
        print(f"| {os.path.basename(f)} | {len(C)} | {tc / 1e6:.3f} | {total(gu) / 1e6:.3f} | {total(both) / 1e6:.3f} | {frac:.3f} |")


if __name__ == "__main__":
    main()
