"""Attention kernel timings (harness shape) and backward grid-cap sweep."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402

D = _native.device()
st = torch.cuda.current_stream().cuda_stream


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


for B, S, H, Dh in [(2048, 16, 4, 64), (2048, 16, 2, 64)]:
    qkv = (torch.randn(B * S, 3 * H * Dh, device="cuda") * 0.5).bfloat16()
    o = torch.empty(B * S, H * Dh, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, S, device="cuda")
    pool = torch.empty(B, H * Dh, device="cuda", dtype=torch.bfloat16)
    gp = torch.randn(B, H * Dh, device="cuda").bfloat16()
    dqkv = torch.empty_like(qkv)
    dbias = torch.zeros(3 * H * Dh, device="cuda")
    fwd = lambda: D.attn_small_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, Dh, qkv.stride(0),  # noqa: E731
                                   o.stride(0), Dh ** -0.5, pool.data_ptr(), pool.stride(0), st)
    bwd = lambda: D.attn_small_bwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), gp.data_ptr(), dqkv.data_ptr(),  # noqa: E731
                                   dbias.data_ptr(), B, S, H, Dh, qkv.stride(0), o.stride(0), Dh ** -0.5,
                                   gp.stride(0), 0, st)
    res = {"fwd": min(t(fwd) for _ in range(3))}
    for cap in (256, 512, 1024, 2048, 4096, 8192):
        D.attn_set_bwd_grid(cap)
        res[f"bwd/{cap}"] = min(t(bwd) for _ in range(3))
    D.attn_set_bwd_grid(0)
    mb = (qkv.numel() * 2 + o.numel() * 2) / 1e6
    print(f"B={B} S={S} H={H} D={Dh} (fwd moves {mb:.0f} MB): " + "  ".join(f"{k} {v:.1f}us" for k, v in res.items()),
          flush=True)
