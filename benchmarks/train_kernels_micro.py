"""Micro-timings of the harness training step's small kernels on their step shapes (B = 2048
sequences x 16 tokens, d_model 768, 4 heads of 64, kp = 72), CUDA-event timed, one JSON line
per measurement:

* ``wgrad``: ``emb_qkv_wgrad`` whole, without the dW_emb part (Ge), without the A-buffer zeroing;
* ``gemm_tn_a``: A = dQKV^T Xp (32768 x 768 by 32768 x 72) over split-K and atomics / workspace;
* ``gemm_tn_o``: dW_o = dZ^T pool (2048 x 16 by 2048 x 256) over split-K."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_tn  # noqa: E402

D = _native.device()
st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731


def t(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        v = s.elapsed_time(e) / iters * 1e3
        best = v if best is None else min(best, v)
    return round(best, 2)


def emit(**kw):
    print(json.dumps(kw), flush=True)


only = sys.argv[1:] or ["wgrad", "gemm_tn_a", "gemm_tn_o", "bwd"]
B, S, Cp = 2048, 16, 16
R, d, kp = 768, 768, 72
if "wgrad" in only:
    A = torch.randn(R, kp, device="cuda")
    We = torch.randn(d, kp, device="cuda")
    Wq = torch.randn(R, d, device="cuda")
    Gq = torch.zeros(R, d, device="cuda")
    Ge = torch.zeros(d, kp, device="cuda")
    Z = torch.zeros(R, kp, device="cuda")
    for name, ge, zz in (("full", Ge, Z), ("no_ge", None, Z), ("no_z", Ge, None), ("gq_only", None, None)):
        us = t(lambda: D.emb_qkv_wgrad(A.data_ptr(), A.stride(0), We.data_ptr(), We.stride(0), Wq.data_ptr(), Wq.stride(0),
                                       Gq.data_ptr(), Gq.stride(0), 0 if ge is None else ge.data_ptr(), kp,
                                       0 if zz is None else zz.data_ptr(), kp, R, d, kp, st()))
        emit(kernel="wgrad", variant=name, us=us)
if "gemm_tn_a" in only:
    M = B * S
    dq = torch.randn(M, 3 * 256, device="cuda").bfloat16()
    xp = torch.randn(M, kp, device="cuda").bfloat16()
    a = torch.zeros(3 * 256, kp, device="cuda")
    for pf in (1, 2):
        D.gemm_tn_set_prefetch(pf)
        for sk in (None, 16, 24, 32, 48, 64):
            for ws in (False, True):
                us = t(lambda: gemm_tn(dq, xp, out=a, accumulate=True, splitk=sk, workspace=ws))
                emit(kernel="gemm_tn_a", pf=pf, splitk=sk, workspace=ws, us=us)
    for shape in ((32768, 768, 768), (32768, 768, 840), (8192, 4096, 4096)):
        M_, N1_, N2_ = shape
        x1 = torch.randn(M_, N1_, device="cuda").bfloat16()
        x2 = torch.randn(M_, N2_, device="cuda").bfloat16()
        o_ = torch.zeros(N1_, N2_, device="cuda")
        for pf in (1, 2):
            D.gemm_tn_set_prefetch(pf)
            us = t(lambda: gemm_tn(x1, x2, out=o_), iters=20)
            emit(kernel="gemm_tn", shape=list(shape), pf=pf, us=us)
        del x1, x2, o_
    D.gemm_tn_set_prefetch(0)
if "gemm_tn_o" in only:
    dzp = torch.randn(B, Cp, device="cuda").bfloat16()
    pool = torch.randn(B, 256, device="cuda").bfloat16()
    go = torch.zeros(Cp, 256, device="cuda")
    for sk in (4, 8, 16, 32):
        us = t(lambda: gemm_tn(dzp, pool, out=go, accumulate=True, splitk=sk))
        emit(kernel="gemm_tn_o", splitk=sk, us=us)
if "bwd" in only:
    # the fused attention backward (token fc_o, dpool formed in-kernel) with / without the
    # in-kernel QKV bias gradient, over workgroups per head
    H, Dh, hd = 4, 64, 256
    qkv = (torch.randn(B * S, 3 * hd, device="cuda") * 0.5).bfloat16()
    lse = torch.randn(B * H * S, device="cuda").abs() + 2
    dqkv = torch.empty(B * S, 3 * hd, device="cuda").bfloat16()
    dbias = torch.zeros(3 * hd, device="cuda")
    dzp = torch.randn(B, Cp, device="cuda").bfloat16()
    wo = torch.randn(Cp, hd, device="cuda").bfloat16()
    for cap in (0, 512, 2048, 4096):
        D.attn_set_bwd_grid(cap)
        for with_db in (True, False):
            us = t(lambda: D.attn_small_bwd(qkv.data_ptr(), 0, lse.data_ptr(), 0, dqkv.data_ptr(),
                                            dbias.data_ptr() if with_db else 0, B, S, H, Dh, qkv.stride(0), hd,
                                            Dh ** -0.5, 0, 0, st(), dz=dzp.data_ptr(), ld_dz=dzp.stride(0),
                                            wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=Cp, dz_scale=1.0 / S))
            emit(kernel="attn_bwd", grid_cap=cap, dbias=with_db, us=us)
    D.attn_set_bwd_grid(0)
