"""Attention forward at the harness shape: pooled only / pooled + fused fc_o logits /
with the per-token output stored, to price each part of the kernel."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402

D = _native.device()
st = torch.cuda.current_stream().cuda_stream


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


B, S, H, Dh = 2048, 16, 4, 64
qkv = (torch.randn(B * S, 3 * H * Dh, device="cuda") * 0.5).bfloat16()
o = torch.empty(B * S, H * Dh, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H, S, device="cuda")
pool = torch.empty(B, H * Dh, device="cuda", dtype=torch.bfloat16)
wo = (torch.randn(16, H * Dh, device="cuda") * 0.1).bfloat16()
zp = torch.empty(B, 16, device="cuda")
bo = torch.randn(16, device="cuda")
sc = Dh ** -0.5
fc = dict(wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16, zp=zp.data_ptr(), ld_zp=zp.stride(0), bo=bo.data_ptr())
res = {
    "pool": t(lambda: D.attn_small_fwd(qkv.data_ptr(), 0, lse.data_ptr(), B, S, H, Dh, qkv.stride(0), H * Dh, sc,
                                       pool.data_ptr(), pool.stride(0), st)),
    "pool+fc_o": t(lambda: D.attn_small_fwd(qkv.data_ptr(), 0, lse.data_ptr(), B, S, H, Dh, qkv.stride(0), H * Dh, sc,
                                            pool.data_ptr(), pool.stride(0), st, **fc)),
    "O+pool": t(lambda: D.attn_small_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, Dh, qkv.stride(0),
                                         o.stride(0), sc, pool.data_ptr(), pool.stride(0), st)),
    "read qkv (sum)": t(lambda: qkv.sum(dtype=torch.float32)),
    "copy qkv third": t(lambda: o.copy_(qkv[:, : H * Dh])),
}
print("  ".join(f"{k} {v:.1f}us" for k, v in res.items()), flush=True)
