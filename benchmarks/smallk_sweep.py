"""Sweep the small-K GEMM kernel's N slice and grid cap against k128 and hipBLASLt."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

D = _native.device()


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for M, N, K in [(32768, 768, 72), (32768, 768, 128), (32768, 384, 72)]:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = (a @ b.T).float()
    res = {}
    for rnd in range(3):
        for bn in (128, 256):
            for grid in (512, 1024, 2048, 4096):
                D.gemm_set_smallk(bn, grid)
                gemm_nt(a, b, out=c)
                if rnd == 0:
                    assert (c.float() - ref).abs().max().item() < 0.1, (bn, grid)
                res.setdefault(f"sk{bn}/g{grid}", []).append(t(lambda: gemm_nt(a, b, out=c)))
        D.gemm_set_smallk(0, 0)
        res.setdefault("k128", []).append(t(lambda: gemm_nt(a, b, out=c)))
        res.setdefault("hipblaslt", []).append(t(lambda: torch.matmul(a, b.T, out=c)))
    D.gemm_set_smallk(128, 0)
    print(f"{M}x{N}x{K}: " + "  ".join(f"{k} {sorted(v)[1]:.1f}us" for k, v in res.items()), flush=True)
