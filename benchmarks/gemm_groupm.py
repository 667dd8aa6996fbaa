"""Tile order of the pair-slot ring: group-M rows (gemm_set_w4_group_m) swept on the Llama
forward shapes, interleaved rounds, median; hipBLASLt for reference.  One JSON line per
shape.  ROUTE=dW: the K-major weight-gradient form (gemm_ring ta = tb = True, operands
[K, M] and [K, N]); ROUTE=dX: K-major B (gemm_ring tb = True, B stored [K, N])."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt, gemm_ring  # noqa: E402


def t_ms(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


D = _native.device()
groups = [int(v) for v in os.environ.get("GROUPS", "2,4,8,16").split(",")]
for shp in os.environ.get("SHAPES", "4096x28672x4096,4096x14336x4096,4096x4096x14336").split(","):
    M, N, K = (int(v) for v in shp.split("x"))
    route = os.environ.get("ROUTE", "nt")
    ta, tb = route == "dW", route in ("dW", "dX")
    a = (torch.rand(*((K, M) if ta else (M, K)), device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(*((K, N) if tb else (N, K)), device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ours = (lambda: gemm_ring(a, b, ta, tb, out=c)) if route != "nt" else (lambda: gemm_nt(a, b, out=c))
    lib = lambda: torch.matmul(a.T if ta else a, b if tb else b.T, out=c)  # noqa: E731
    res = {g: [] for g in groups}
    res["hipblaslt"] = []
    for _ in range(5):
        for g in groups:
            D.gemm_set_w4_group_m(g)
            res[g].append(t_ms(ours))
        res["hipblaslt"].append(t_ms(lib))
    D.gemm_set_w4_group_m(8)
    blas = statistics.median(res["hipblaslt"])
    out = {"shape": shp, "route": route, "hipblaslt_ms": round(blas, 4)}
    for g in groups:
        ms = statistics.median(res[g])
        out[f"group_m{g}"] = {"ms": round(ms, 4), "vs_hipblaslt": round(blas / ms, 3)}
    print(json.dumps(out), flush=True)
