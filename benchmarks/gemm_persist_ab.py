"""The pair-slot ring GEMM with and without the persistent grid (ring schedule bit 0: one
workgroup per CU walking its tiles, the next tile's first pairs loaded under the epilogue),
interleaved rounds, median, hipBLASLt for reference; forward NT shapes.  One JSON line per shape.

    python benchmarks/gemm_persist_ab.py [--rounds 5] [--shapes MxNxK,...]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402


def t_ms(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--shapes", default="4096x28672x4096,4096x4096x14336,4096x14336x4096")
args = ap.parse_args()
D = _native.device()
BASE = int(os.environ.get("CCMPI_RING_SCHED", str(8 | 16384)))  # the default ring schedule
for shp in args.shapes.split(","):
    M, N, K = (int(v) for v in shp.split("x"))
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = None
    res = {"default": [], "persist": [], "hipblaslt": []}
    for _ in range(args.rounds):
        for mode in ("default", "persist"):
            D.gemm_set_ring_sched(BASE | 1 if mode == "persist" else BASE)
            res[mode].append(t_ms(lambda: gemm_nt(a, b, out=c)))
            if ref is None:
                ref = c.clone()
            elif mode == "persist":
                assert torch.equal(c, ref), "persistent grid changed the result"
        res["hipblaslt"].append(t_ms(lambda: torch.matmul(a, b.T, out=c)))
    D.gemm_set_ring_sched(BASE)
    blas = statistics.median(res["hipblaslt"])
    out = {"shape": shp, "hipblaslt_ms": round(blas, 4)}
    for m in ("default", "persist"):
        ms = statistics.median(res[m])
        out[m] = {"ms": round(ms, 4), "vs_hipblaslt": round(blas / ms, 3)}
    print(json.dumps(out), flush=True)
