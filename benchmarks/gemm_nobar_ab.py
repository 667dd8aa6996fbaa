"""Upper bound of the pair ring's barrier skew: the forward NT GEMM with
its odd-phase barrier (default) against the same kernel with the barrier reduced to each
wave's own waits (``gemm_set_pair_nobar(1)``: races, wrong results -- timing only) and
hipBLASLt, in interleaved rounds.  One JSON line per shape.

    python benchmarks/gemm_nobar_ab.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--shapes", default="4096x4096x14336,4096x28672x4096,4096x14336x4096")
args = ap.parse_args()
D = _native.device()


def time_ms(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(args.iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / args.iters


for shp in args.shapes.split(","):
    M, N, K = (int(v) for v in shp.split("x"))
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    names = {0: "ring", 1: "ring_nobarrier", 2: "ring_nodmawait", 3: "ring_neither"}
    res = {v: [] for v in names.values()}
    res["hipblaslt"] = []
    for _ in range(args.rounds):
        for k, name in names.items():
            D.gemm_set_pair_nobar(k)
            res[name].append(time_ms(lambda: gemm_nt(a, b, out=c)))
        D.gemm_set_pair_nobar(0)
        res["hipblaslt"].append(time_ms(lambda: torch.matmul(a, b.T, out=c)))
    out = {"shape": shp}
    for k, v in res.items():
        ms = statistics.median(v)
        out[k] = {"ms": round(ms, 4), "TF": round(2 * M * N * K / ms / 1e9, 1)}
    for k in names.values():
        out[k]["vs_hipblaslt"] = round(out["hipblaslt"]["ms"] / out[k]["ms"], 3)
    print(json.dumps(out), flush=True)
