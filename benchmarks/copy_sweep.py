"""Device-to-device copy bandwidth sweep: the single-rank all-reduce of bench.py
is a 1 GiB copy, so this is the kernel behind the N = 1 headline.  Variants of
`k_copy_v` (vectors in flight per lane, non-temporal hints, grid-stride vs
contiguous slices) x grid sizes, against the runtime's blit (hipMemcpyAsync).
Interleaved rounds, median reported.

    python benchmarks/copy_sweep.py [--mib 1024] [--rounds 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402

NAMES = {0: "u4_nt", 1: "u8_nt", 2: "u4_plain", 3: "u4_ntload", 4: "u4_ntstore", 5: "u4_nt_contig",
         6: "u8_nt_contig", 7: "u2_nt", 8: "u16_nt", 9: "u2_nt_contig", 10: "u4_ntstore_contig",
         11: "u4_plain_contig", 12: "u1_nt_contig"}
CONTIG = (5, 6, 9, 10, 11, 12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--allreduce", action="store_true", help="also time the single-rank all-reduce path")
    ap.add_argument("--variants", default=",".join(map(str, CONTIG)), help="contiguous-slice variants to sweep")
    ap.add_argument("--grids", default="8192,16384,32768,65536,131072")
    args = ap.parse_args()
    args.grids = [int(g) for g in args.grids.split(",")]
    contig = [int(v) for v in args.variants.split(",")]
    D = _native.device()
    n = args.mib << 20
    x = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    variants = {"blit": lambda: y.copy_(x)}
    if args.allreduce:  # the bench.py path: symmetric-heap buffers through DeviceGroup.allreduce
        from collective_communication_mpi_amd import MPI, Communicator

        dev = Communicator(MPI.COMM_WORLD).dev
        xs, ys = dev.empty(n // 4, torch.float32), dev.empty(n // 4, torch.float32)
        xs.copy_(x.view(torch.float32))
        xs.fill_(1.0)
        variants["allreduce_heap"] = lambda: dev.allreduce(xs, ys, "SUM", "twoshot")
        variants["u1_nt_contig_heap"] = lambda: D.copy_variant(xs.data_ptr(), ys.data_ptr(), n, 12, n // 4096, st)
    variants["u4_nt_g4096"] = lambda: D.copy_variant(x.data_ptr(), y.data_ptr(), n, 0, 4096, st)
    for v in contig:
        for g in args.grids:
            variants[f"{NAMES[v]}_g{g}"] = (lambda v=v, g=g: D.copy_variant(x.data_ptr(), y.data_ptr(), n, v, g, st))
    for k, f in variants.items():  # correctness
        if "heap" in k:
            continue
        y.zero_()
        f()
        torch.cuda.synchronize()
        assert torch.equal(x, y), k
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for k, f in variants.items():
            f()
            s.record()
            for _ in range(args.iters):
                f()
            e.record()
            e.synchronize()
            res[k].append(s.elapsed_time(e) / args.iters)
    out = {}
    for k, ts in res.items():
        ts.sort()
        ms = ts[len(ts) // 2]
        out[k] = {"ms": round(ms, 4), "algbw_GBps": round(n / ms / 1e6, 1)}
    for k, v in sorted(out.items(), key=lambda kv: kv[1]["ms"]):
        print(f"{k:>22}: {v['ms']:.4f} ms  {v['algbw_GBps']:.0f} GB/s", flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
