"""Kernel-variant sweep on the harness QKV projection shapes (bias epilogue, bf16 out):
TP = 1 (32768 x 768 x 768) and TP = 2 (32768 x 384 x 768), against hipBLASLt."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

D = _native.device()


def t(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best


def reset():
    D.gemm_set_kernel(0)
    

VARIANTS = {
    "auto": lambda: None,
    "k128": lambda: D.gemm_set_kernel(1),
    "k256x256": lambda: D.gemm_set_kernel(2),
    "k256x128": lambda: D.gemm_set_kernel(3),
    "k256x192": lambda: D.gemm_set_kernel(4),
}

for M, N, K in [(32768, 768, 768), (32768, 384, 768), (4096, 4096, 4096), (8192, 8192, 1024)]:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) / 16).bfloat16()
    bias = torch.randn(N, device="cuda")
    ref = a.float() @ w.float().t() + bias
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = []
    for name, setup in VARIANTS.items():
        reset()
        setup()
        try:
            c.zero_()
            gemm_nt(a, w, out=c, bias=bias)
            torch.cuda.synchronize()
            err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
            if err > 2e-2:
                res.append(f"{name}:BAD({err:.2e})")
                continue
            us = t(lambda: gemm_nt(a, w, out=c, bias=bias))
            res.append(f"{name}:{us:.1f}")
        except Exception as e:  # noqa: BLE001 - illegal variant for the shape
            res.append(f"{name}:n/a({str(e)[:30]})")
    reset()
    wt = w.t()
    res.append(f"hipblaslt:{t(lambda: torch.addmm(bias.bfloat16(), a, wt, out=c)):.1f}")
    print(f"{M}x{N}x{K}: " + "  ".join(res), flush=True)
