"""Tile order of the pair-slot ring: group-M rows (gemm_set_w4_group_m) swept on the Llama
forward shapes, interleaved rounds, median; hipBLASLt for reference.  One JSON line per
shape."""
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


D = _native.device()
groups = [int(v) for v in os.environ.get("GROUPS", "2,4,8,16").split(",")]
for shp in os.environ.get("SHAPES", "4096x28672x4096,4096x14336x4096,4096x4096x14336").split(","):
    M, N, K = (int(v) for v in shp.split("x"))
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {g: [] for g in groups}
    res["hipblaslt"] = []
    for _ in range(5):
        for g in groups:
            D.gemm_set_w4_group_m(g)
            res[g].append(t_ms(lambda: gemm_nt(a, b, out=c)))
        res["hipblaslt"].append(t_ms(lambda: torch.matmul(a, b.T, out=c)))
    D.gemm_set_w4_group_m(8)
    blas = statistics.median(res["hipblaslt"])
    out = {"shape": shp, "hipblaslt_ms": round(blas, 4)}
    for g in groups:
        ms = statistics.median(res[g])
        out[f"group_m{g}"] = {"ms": round(ms, 4), "vs_hipblaslt": round(blas / ms, 3)}
    print(json.dumps(out), flush=True)
