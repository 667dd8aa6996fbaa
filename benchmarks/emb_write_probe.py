"""Where does the patch-embedding GEMM's time go?  Compares, on the harness
shape (32768 x 768 output, K = 72), the small-K GEMM writing into the padded
[h | xp] rows against plain write kernels of the same bytes, and sweeps the
small-K kernel's N slice / grid."""
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


M, N, K, LD = 32768, 768, 72, 896
hx = torch.zeros(M, LD, device="cuda", dtype=torch.bfloat16)
h = hx[:, :N]
xp = hx[:, N:N + K]
xp.copy_((torch.rand(M, K, device="cuda") * 2 - 1).bfloat16())
w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
flat = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
res = {
    "fill_contig_50MB": t(lambda: flat.fill_(1.0)),
    "fill_strided_h": t(lambda: h.fill_(1.0)),
    "copy_contig_50MB": t(lambda: flat.copy_(h)),
    "gemm_default_hx": t(lambda: gemm_nt(xp, w, out=h)),
    "gemm_default_contig": t(lambda: gemm_nt(xp.contiguous(), w, out=flat)),
    "hipblaslt_contig": t(lambda: torch.matmul(xp, w.T, out=flat)),
}
for bn in (128, 256):
    for grid in (256, 512, 768, 1024, 1536, 2048, 3072, 4096):
        D.gemm_set_smallk(bn, grid)
        res[f"sk{bn}_g{grid}"] = t(lambda: gemm_nt(xp, w, out=h))
D.gemm_set_smallk(0, 0)
res["k128_hx"] = t(lambda: gemm_nt(xp, w, out=h))
D.gemm_set_smallk(128, 0)
mb = M * N * 2 / 1e6
for k, v in res.items():
    print(f"{k:24s} {v:7.2f} us  {mb / v:6.2f} TB/s (output bytes)", flush=True)
