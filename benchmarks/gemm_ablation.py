"""Ablations of the 256x256 ping-pong GEMM (interleaved rounds, one process).

bits: 1 = no vmcnt waits (results WRONG; isolates DMA-latency stalls), 2 = no
s_setprio, 4 = no ping-pong stagger.  Prints TF/s per variant and shape.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

D = _native.device()
D.gemm_set_kernel(2)
shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 4096, 14336)]
for M, N, K in shapes:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    res = {}
    for _ in range(5):
        for e in (0, 1, 2, 4, 6):
            D.gemm_set_ablation(e)
            gemm_nt(a, b, out=c)
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(10):
                gemm_nt(a, b, out=c)
            t.record()
            t.synchronize()
            res.setdefault(e, []).append(s.elapsed_time(t) / 10)
    D.gemm_set_ablation(0)
    print(f"{M}x{N}x{K}: " + "  ".join(f"exp{e} {fl / sorted(v)[2] / 1e9:.0f}TF" for e, v in res.items()), flush=True)
