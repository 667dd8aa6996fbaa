"""Small-K (patch embedding) GEMM with plain vs non-temporal bf16 stores, alone and
followed by the QKV GEMM that reads its output (harness shapes, [h | xp] layout)."""
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
h, xp = hx[:, :N], hx[:, N:N + K]
xp.copy_((torch.rand(M, K, device="cuda") * 2 - 1).bfloat16())
w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
wq = ((torch.rand(768, N, device="cuda") * 2 - 1) / 16).bfloat16()
bq = torch.randn(768, device="cuda")
qkv = torch.empty(M, 768, device="cuda", dtype=torch.bfloat16)
ref = xp.float() @ w.float().t()
for nt in (False, True, False, True):
    D.gemm_set_smallk_nt(nt)
    gemm_nt(xp, w, out=h)
    torch.cuda.synchronize()
    assert ((h.float() - ref).abs().max() < 0.05), nt
    a = t(lambda: gemm_nt(xp, w, out=h))
    b = t(lambda: (gemm_nt(xp, w, out=h), gemm_nt(h, wq, out=qkv, bias=bq)))
    print(f"nt={int(nt)}: smallk {a:.1f} us   smallk+qkv {b:.1f} us", flush=True)
