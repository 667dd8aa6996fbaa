"""LDS-ring NT GEMM variants vs hipBLASLt on the Llama-3-8B MLP shapes.

    python benchmarks/gemm_ps_ab.py [--rounds 5] [--scheds 8,16392]

Variants (``gemm_set_ring_sched``: bit 3 the ring, bit 14 pair slots, bit 0 persistent
grid, bit 15 long K on the ring too, bit 13 the whole-line ablation) and hipBLASLt
(torch.matmul) are timed in interleaved rounds in one process (median of per-round
medians), bf16 in / out, uniform random operands.  One JSON line per shape."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

SHAPES = ["4096x4096x14336", "4096x28672x4096", "4096x4096x28672", "4096x14336x4096"]


def time_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--shapes", default=",".join(SHAPES))
ap.add_argument("--scheds", default="8,16392")
args = ap.parse_args()
D = _native.device()
scheds = [int(v) for v in args.scheds.split(",")]
for shp in args.shapes.split(","):
    M, N, K = (int(v) for v in shp.split("x"))
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = (a.float() @ b.float().T)
    res = {f"ring{s}": [] for s in scheds}
    res["hipblaslt"] = []
    errs = {}
    for _ in range(args.rounds):
        for s in scheds:
            D.gemm_set_ring_sched(s)
            res[f"ring{s}"].append(time_ms(lambda: gemm_nt(a, b, out=c), args.iters))
            errs[f"ring{s}"] = float(((c.float() - ref).abs().max() / ref.abs().max()).item())
        res["hipblaslt"].append(time_ms(lambda: torch.matmul(a, b.T, out=c), args.iters))
    D.gemm_set_ring_sched(8 | 16384)
    fl = 2 * M * N * K
    out = {"shape": shp}
    for k, v in res.items():
        ms = statistics.median(v)
        out[k] = {"ms": round(ms, 4), "TF": round(fl / ms / 1e9, 1)}
    for s in scheds:
        out[f"ring{s}"]["vs_hipblaslt"] = round(out["hipblaslt"]["ms"] / out[f"ring{s}"]["ms"], 3)
        out[f"ring{s}"]["max_rel_err"] = round(errs[f"ring{s}"], 5)
    print(json.dumps(out), flush=True)
