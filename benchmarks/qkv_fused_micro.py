"""Fused QKV + attention + token fc_o kernel (k_qkv_attn16_fwd) in isolation: event-timed
per mode (patch rows vs images, inference vs training stores, token mean vs z rows) and
persistent grid size, against the unfused QKV GEMM + attention kernel.  One JSON line per
configuration.  Usage: python benchmarks/qkv_fused_micro.py [--iters N] [--only MODE]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops.kernels import gemm_nt  # noqa: E402


def timed(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--only", default="")
    ap.add_argument("--grid", type=int, default=0, help="only this persistent grid size")
    ap.add_argument("--train", type=int, default=-1, help="0/1: only inference / training stores")
    args = ap.parse_args()
    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    B, H, D, S, kp = args.B, args.H, 64, 16, 72
    HD = H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.rand(B, 784, device="cuda", generator=g)
    xp = torch.empty(B * S, kp, device="cuda", dtype=torch.bfloat16)
    dev.patchify(img.data_ptr(), xp.data_ptr(), B, 28, 7, kp, st, kp)
    w = (torch.randn(3 * HD, kp, device="cuda", generator=g) / kp ** 0.5).bfloat16()
    bq = torch.randn(3 * HD, device="cuda", generator=g) * 0.1
    wo = (torch.randn(16, HD, device="cuda", generator=g) * 0.1).bfloat16()
    bo = torch.randn(16, device="cuda", generator=g)
    qkv = torch.empty(B * S, 3 * HD, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, S, device="cuda")
    pool = torch.empty(B, HD, device="cuda", dtype=torch.bfloat16)
    z = torch.empty(B * S, 16, device="cuda")
    zm = torch.empty(B, 16, device="cuda")
    common = dict(lse=lse.data_ptr(), B=B, S=S, Hl=H, D=D, scale=D ** -0.5, pool=pool.data_ptr(),
                  ld_pool=pool.stride(0), wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16, bo=bo.data_ptr(), ld_zt=16,
                  zrows=0, zpush=[], stream=st, ld_xq=kp, kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(),
                  ld_qkv=qkv.stride(0))

    def fused(mode, train, mean):
        kw = dict(common)
        kw.update(pool=pool.data_ptr() if train else 0,  # (the model passes pool only for a backward)
                  xq=0 if mode == "img" else xp.data_ptr(), img=img.data_ptr() if mode == "img" else 0,
                  xq_out=xp.data_ptr() if (mode == "img" and train) else 0, qkv_out=qkv.data_ptr() if train else 0,
                  ztok=0 if mean else z.data_ptr(), zmean=zm.data_ptr() if mean else 0)
        return lambda: dev.attn_qkv_fwd(**kw)

    def unfused():
        gemm_nt(xp, w, out=qkv, bias=bq)
        dev.attn_small_fwd(qkv.data_ptr(), 0, lse.data_ptr(), B, S, H, D, qkv.stride(0), HD, D ** -0.5,
                           pool.data_ptr(), pool.stride(0), st, wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16,
                           bo=bo.data_ptr(), ztok=z.data_ptr(), ld_zt=16)

    rows = []
    if not args.only or args.only == "unfused":
        rows.append(dict(kernel="unfused", us=timed(unfused, args.iters)))
    for cap in ((args.grid,) if args.grid else (256, 512, 1024, 2048)):
        dev.attn_set_qkv_grid(cap)
        for mode in ("rows", "img"):
            for train in ((bool(args.train),) if args.train >= 0 else (False, True)):
                for mean in (False, True):
                    if args.only and args.only != mode:
                        continue
                    rows.append(dict(kernel="fused", mode=mode, train=train, mean=mean, grid=cap,
                                     us=timed(fused(mode, train, mean), args.iters)))
    dev.attn_set_qkv_grid(0)
    for r in rows:
        r.update(B=B, H=H)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
