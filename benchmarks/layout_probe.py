"""Activation layout of the harness forward/backward: the fused [h | xp] rows (ld 896)
against separate contiguous h / xp buffers, timing the three kernels that touch them:
patch-embedding GEMM (xp -> h), QKV GEMM (h -> qkv), A = dQKV^T xp (TN GEMM)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_nt, gemm_tn  # noqa: E402


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


M, d, kp = 32768, 768, 72
w_emb = ((torch.rand(d, kp, device="cuda") * 2 - 1) / 8).bfloat16()
w_qkv = ((torch.rand(768, d, device="cuda") * 2 - 1) / 16).bfloat16()
b_qkv = torch.randn(768, device="cuda")
qkv = torch.empty(M, 768, device="cuda", dtype=torch.bfloat16)
dqkv = torch.randn(M, 768, device="cuda").bfloat16()
a = torch.zeros(768, kp, device="cuda")
src = (torch.rand(M, kp, device="cuda") * 2 - 1).bfloat16()
layouts = {}
hx = torch.zeros(M, 896, device="cuda", dtype=torch.bfloat16)
layouts["hx896"] = (hx[:, :d], hx[:, d:d + kp])
layouts["contig_xp72"] = (torch.zeros(M, d, device="cuda", dtype=torch.bfloat16),
                          torch.zeros(M, kp, device="cuda", dtype=torch.bfloat16))
layouts["contig_xp128"] = (torch.zeros(M, d, device="cuda", dtype=torch.bfloat16),
                           torch.zeros(M, 128, device="cuda", dtype=torch.bfloat16)[:, :kp])
for name, (h, xp) in layouts.items():
    xp.copy_(src)
    e = t(lambda: gemm_nt(xp, w_emb, out=h))
    q = t(lambda: gemm_nt(h, w_qkv, out=qkv, bias=b_qkv))
    eq = t(lambda: (gemm_nt(xp, w_emb, out=h), gemm_nt(h, w_qkv, out=qkv, bias=b_qkv)))
    ag = t(lambda: gemm_tn(dqkv, xp, out=a, accumulate=True, workspace=False))
    print(f"{name:14s} emb {e:5.1f}  qkv {q:5.1f}  emb+qkv {eq:5.1f}  A {ag:5.1f} us", flush=True)
