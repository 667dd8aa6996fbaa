"""Is the narrow-N, K=768 GEMM epilogue (store) bound?  128x128 kernel with and
without its epilogue, bf16 vs fp32 output."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

D = _native.device()
D.gemm_set_kernel(1)


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


for M, N, K in [(32768, 768, 768), (32768, 768, 2304), (8192, 8192, 1024)]:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    res = {}
    for _ in range(3):
        for od in (torch.bfloat16, torch.float32):
            c = torch.empty(M, N, device="cuda", dtype=od)
            for ab in (0, 8, 16):
                D.gemm_set_ablation(ab & 8)
                D.gemm_set_direct_epilogue(ab != 16)
                tag = {0: "-fast", 8: "-noepi", 16: "-staged"}[ab]
                res.setdefault(f"{'bf16' if od == torch.bfloat16 else 'fp32'}{tag}", []).append(
                    t(lambda: gemm_nt(a, b, out=c, splitk=1)))
            D.gemm_set_direct_epilogue(True)
    D.gemm_set_ablation(0)
    fl = 2 * M * N * K
    print(f"{M}x{N}x{K}: " + "  ".join(f"{k} {sorted(v)[1]:.1f}us ({fl / sorted(v)[1] / 1e6:.0f}TF)" for k, v in res.items()),
          flush=True)
x = torch.empty(32768 * 768, dtype=torch.bfloat16, device="cuda")
print(f"fill 50MB bf16: {t(lambda: x.fill_(1.0)):.1f}us", flush=True)
