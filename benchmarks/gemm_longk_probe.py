"""Why long K runs slower on the ring kernels (4096^2 x 28672 at ~0.83x hipBLASLt, against
0.94x for 4096^2 x 14336 with the same 256 tiles): the same K = 14336 GEMM on contiguous
operands and on views with the long-K row stride (28672), and the full long-K GEMM.  If
the strided views are slow, the row stride (address translation / cache sets) is the cause,
not the loop length.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402


def time_ms(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


M = N = 4096
a_long = (torch.rand(M, 28672, device="cuda") * 2 - 1).bfloat16()
b_long = (torch.rand(N, 28672, device="cuda") * 2 - 1).bfloat16()
a_half = a_long[:, :14336].contiguous()
b_half = b_long[:, :14336].contiguous()
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
res = {}
for name, (a, b) in {"k14336_contig": (a_half, b_half), "k14336_stride28672": (a_long[:, :14336], b_long[:, :14336]),
                     "k28672": (a_long, b_long)}.items():
    K = a.shape[1]
    own = time_ms(lambda: gemm_nt(a, b, out=c))
    blas = time_ms(lambda: torch.matmul(a, b.T, out=c))
    res[name] = {"own_ms": round(own, 4), "own_TF": round(2 * M * N * K / own / 1e9, 1),
                 "hipblaslt_ms": round(blas, 4), "vs_hipblaslt": round(blas / own, 3)}
print(json.dumps(res), flush=True)
