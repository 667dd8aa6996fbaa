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
    # (50 untimed launches: with 5, whichever configuration ran first after a switch read
    # 0.3-1 us slower than the same launch timed later -- profiles/r6_attn micro_v1x)
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def trace_phases(fused, mode, train, mean, cap, npairs):
    """Launch once more with phase stamps; medians over waves of each phase (shader clocks).
    Stamp k: 0 entry, 1 loop entry (prologue done), per iteration j < 4 at 2 + 5 j: start
    (X in registers), +1 q|k|v projected, +2 z formed, +3 before the workgroup barrier (image
    mode: after the DMA wait and the next X build), +4 epilogue stored; 31 kernel end."""
    import numpy as np

    nw = 8  # waves per workgroup of k_qkv_attn16_fwd (attn_mfma.hip kQkvWaves)
    waves = min(cap, (npairs + nw - 1) // nw) * nw
    ts = torch.zeros(waves * 32, dtype=torch.int64, device="cuda")
    fused(mode, train, mean, ts.data_ptr())()
    torch.cuda.synchronize()
    t = ts.view(waves, 32).cpu().numpy().astype(np.int64)
    t = t[t[:, 0] != 0]
    out = {"waves": int(len(t)), "prologue": int(np.median(t[:, 1] - t[:, 0]))}
    # inside the prologue: 24 W_h loads issued, 25 tail fragments + biases in, 26 (image mode)
    # every load and both images' DMA in, 27 first X built
    pro = {"w_issue": (0, 24), "w_arrive": (24, 25), "dma_wait": (25, 26), "build_x0": (26, 27), "to_loop": (27, 1),
           "first_loads": (0, 28), "w_dma": (28, 29), "w_frags": (29, 24)}
    out["prologue_parts"] = {k: int(np.median(t[:, b] - t[:, a])) for k, (a, b) in pro.items()
                             if (t[:, a] != 0).all() and (t[:, b] != 0).all()}
    names = ["proj", "attn_z", "dma_wait_build", "barrier_epilogue", "to_next"]
    for j in range(4):
        b = 2 + 5 * j
        ok = t[:, b] != 0
        if not ok.any():
            break
        tj = t[ok]
        ph = {"from_prev": int(np.median(tj[:, b] - (tj[:, 1] if j == 0 else tj[:, b - 1])))}
        for k, nm in enumerate(names[:4]):
            ph[nm] = int(np.median(tj[:, b + k + 1] - tj[:, b + k]))
        out[f"it{j}"] = ph
    out["tail"] = int(np.median(t[:, 31] - np.max(np.where(t[:, 2:22] != 0, t[:, 2:22], 0), axis=1)))
    out["wave_span_median"] = int(np.median(t[:, 31] - t[:, 0]))
    out["kernel_span"] = int(t[:, 31].max() - t[:, 0].min())
    out["start_skew"] = int(np.percentile(t[:, 0], 95) - t[:, 0].min())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--only", default="")
    ap.add_argument("--grid", type=int, default=0, help="only this persistent grid size")
    ap.add_argument("--train", type=int, default=-1, help="0/1: only inference / training stores")
    ap.add_argument("--nolse", action="store_true", help="inference without the lse store (lse = null)")
    ap.add_argument("--fold", action="store_true",
                    help="image mode also folds the next W_eff in-kernel (the pipelined plan's fold tail, d = 768)")
    ap.add_argument("--trace", action="store_true",
                    help="one extra launch with phase stamps (AttnArgs.tstamp): per-phase shader-clock medians")
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

    wq32 = torch.randn(3 * HD, 768, device="cuda", generator=g) / 768 ** 0.5
    we32 = torch.randn(768, kp, device="cuda", generator=g) / 8
    wnext = torch.empty(3 * HD, kp, device="cuda", dtype=torch.bfloat16)

    def fused(mode, train, mean, tstamp=0):
        kw = dict(common)
        if args.fold and mode == "img":
            kw.update(fold_wq=wq32.data_ptr(), ld_fold_wq=768, fold_we=we32.data_ptr(), ld_fold_we=kp,
                      fold_out=wnext.data_ptr(), ld_fold_out=kp, fold_R=3 * HD, fold_d=768)
        if args.nolse and not train:
            kw["lse"] = 0
        if tstamp:
            kw["tstamp"] = tstamp
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
                    fold = bool(args.fold and mode == "img")
                    # with the fold: the fold-aware block schedule on (1) and off (0), interleaved
                    for sched in ((1, 0) if fold else (-1,)):
                        dev.attn_set_qkv_fold_sched(sched)
                        rows.append(dict(kernel="fused", mode=mode, train=train, mean=mean, grid=cap,
                                         us=timed(fused(mode, train, mean), args.iters), nolse=args.nolse,
                                         fold=fold, **({"fold_sched": sched} if fold else {})))
                        if args.trace:
                            rows[-1]["phases"] = trace_phases(fused, mode, train, mean, cap, B * H)
                    dev.attn_set_qkv_fold_sched(-1)
    dev.attn_set_qkv_grid(0)
    for r in rows:
        r.update(B=B, H=H)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
