"""GEMM A/B: our 128x128 kernel vs the 256x256 ping-pong kernel vs hipBLASLt
(torch.matmul), bf16 in, bf16 out, uniform random operands.  Variants are timed
in interleaved rounds inside one process (median over rounds of the per-round
median), so clock drift hits all of them alike.

    python benchmarks/gemm_bench.py [--rounds 5] [--shapes 4096x4096x4096,...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

DEFAULT = ["4096x4096x4096", "8192x8192x8192", "32768x768x768", "32768x384x768", "16384x4096x4096",
           "8192x14336x4096", "8192x4096x14336", "32768x2304x768"]


def time_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default=",".join(DEFAULT))
    ap.add_argument("--json", default="")
    ap.add_argument("--all", action="store_true", help="also the 128x128 and 256x192 kernels")
    ap.add_argument("--w4", default="0:8,1:8,3:8",
                    help="four-wave kernel variants sched:group_m (sched bit 0 persistent, bit 1 MFMA-first)")
    args = ap.parse_args()
    D = _native.device()
    out = []
    for shp in args.shapes.split(","):
        M, N, K = (int(v) for v in shp.split("x"))
        a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        iters = max(3, int(2e12 / fl))

        def ours(mode):
            def f():
                D.gemm_set_kernel(mode)
                gemm_nt(a, b, out=c)
            return f

        def w4(sched, gm):
            def f():
                D.gemm_set_kernel(5)
                D.gemm_set_w4_sched(sched)
                D.gemm_set_w4_group_m(gm)
                gemm_nt(a, b, out=c)
            return f

        variants = {"k256": ours(2)}
        for v in args.w4.split(","):
            if v:
                sc, gm = (int(x) for x in v.split(":"))
                variants[f"w4s{sc}g{gm}"] = w4(sc, gm)
        variants.update({"auto": ours(0), "hipblaslt": lambda: torch.matmul(a, b.T, out=c)})
        if args.all:
            variants.update({"k128": ours(1), "k256x192": ours(4)})
        # correctness of both kernels on this shape against hipBLASLt
        ref = (a @ b.T).float()
        # (w4 schedules with bit 5/6 set are timing ablations with wrong results)
        abl = {f"w4s{v.split(':')[0]}g{v.split(':')[1]}" for v in args.w4.split(",") if v and int(v.split(":")[0]) & 96}
        for k in [v for v in variants if v not in ("auto", "hipblaslt") and v not in abl]:
            variants[k]()
            err = (c.float() - ref).abs().max().item()
            assert err < 0.05 * K ** 0.5, f"{k} {shp}: max err {err}"
        res = {k: [] for k in variants}
        for _ in range(args.rounds):
            for k, f in variants.items():
                res[k].append(time_ms(f, iters))
        D.gemm_set_kernel(0)
        row = {"shape": shp}
        for k, ts in res.items():
            ts.sort()
            ms = ts[len(ts) // 2]
            row[k] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
        out.append(row)
        print(f"{shp:>20}: " + "  ".join(f"{k} {v['ms']:.3f} ms {v['tflops']:.0f} TF" for k, v in row.items()
                                         if k != "shape"), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
