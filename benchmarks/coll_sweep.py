"""Collective-kernel sweep with bytes/time accounting.

    scripts/mpirun -n 4 python benchmarks/coll_sweep.py --ops allreduce --max-mb 256 --out gpurun_out/cs4.jsonl
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/coll_sweep.py --ops all

For every (op, algorithm, CTA budget, size) the sweep

* checks the result once (rank-valued inputs: SUM results are exact),
* times ``--iters`` back-to-back calls between two hipEvents on every rank
  (the kernels synchronise the ranks themselves, so back-to-back calls are
  the steady state; the start skew of one barrier is amortised), MAX over ranks,
* reports NCCL-tests algbw/busbw *and* the HBM bytes the kernels really move
  summed over all ranks (``hbm_bytes``: every byte loaded or stored, local or
  through a peer mapping), ``hbm_GBps`` and ``hbm_frac`` against a 6.3 TB/s
  measured HBM ceiling.  With several ranks sharing ONE GPU every byte of
  every rank crosses the same HBM, so ``hbm_frac`` is the efficiency figure
  there; on an xGMI node ``busbw_GBps`` against the link ceiling is.

``size`` follows NCCL-tests: all-reduce = the buffer, all-gather = the
output, reduce-scatter = the input, all-to-all = the per-rank buffer.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

HBM_CEIL = 6.3e12

ap = argparse.ArgumentParser()
ap.add_argument("--ops", default="allreduce", help="comma list of allreduce,allgather,reduce_scatter,alltoall,lastaxis | all")
ap.add_argument("--algos", default="", help="comma list (default: every hand-written algorithm of the op)")
ap.add_argument("--blocks", default="0", help="comma list of per-rank CTA budgets (0 = the group default)")
ap.add_argument("--min-bytes", type=int, default=4096)
ap.add_argument("--max-mb", type=int, default=256)
ap.add_argument("--factor", type=int, default=4, help="size step")
ap.add_argument("--iters", type=int, default=0, help="timed calls per point (0 = size-dependent)")
ap.add_argument("--dtype", default="float32")
ap.add_argument("--out", default="")
args = ap.parse_args()

comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
dev = comm.dev
hc = comm.comm
dt = getattr(torch, args.dtype)
es = torch.empty((), dtype=dt).element_size()
maxb = args.max_mb << 20

ALL_OPS = ["allreduce", "allgather", "reduce_scatter", "alltoall", "lastaxis", "bcast"]
ops = ALL_OPS if args.ops == "all" else args.ops.split(",")
DEFAULT_ALGOS = {
    "allreduce": ["ll", "oneshot", "twoshot", "fanout", "fanout_lds", "push", "reduce_bcast", "ring", "rhd"],
    "allgather": ["direct", "push"],
    "reduce_scatter": ["direct"],
    "alltoall": ["direct", "push", "pairwise"],  # pairwise: same bytes, one peer per round
    "lastaxis": ["gather", "rscatter"],
    "bcast": ["direct", "push"],
}
if not dev.shared_device:
    DEFAULT_ALGOS["allreduce"].append("rccl")
    for k in ("allgather", "reduce_scatter", "alltoall"):
        DEFAULT_ALGOS[k].append("rccl")
if p & (p - 1):
    DEFAULT_ALGOS["allreduce"].remove("rhd")


def hbm_model(op: str, algo: str, S: int) -> float:
    """Bytes read + written by the hand-written kernels, summed over all ranks
    (S as defined in the module docstring)."""
    if op == "allreduce":
        return {
            "oneshot": p * p * S + p * S,            # everyone reads all p buffers, writes S
            "ll": p * (S + 2 * p * S + 2 * p * S + S),  # read S, push 2pS (8 B per 4 B), poll 2pS, write S
            "twoshot": (2 * p - 1) * S + p * S,       # RS: read pS write S; AG: read (p-1)S write (p-1)S
            "fanout": 2 * p * S,                      # every rank reads S (its shard from all), writes S (to all)
            "fanout_lds": 2 * p * S,
            "push": 2 * p * S + 2 * p * S,            # scatter: read pS write pS; reduce+fan-out: same
            "reduce_bcast": (2 * p - 1) * S + p * S,  # root reads pS writes S; p-1 copies of S
            # ring, per rank: RS reads (2p-3)/p S + final 2/p S, writes p/p S; AG copies (p-2)/p S
            "ring": p * (5 * p - 4) / p * S,
            # rhd, per rank: halving pushes (p-1)/p S (read+write) and reduces it (2 reads + 1 write);
            # doubling pushes (p-1)/p S (read + write)
            "rhd": p * 7 * (p - 1) / p * S,
        }.get(algo, 0.0)
    if op == "allgather" and algo == "push":
        return (p + 1) * S                            # every rank reads its S/p block once, writes S
    if op in ("allgather", "alltoall"):
        return 2 * p * S                              # every rank reads S, writes S
    if op == "reduce_scatter":
        return p * S + S                              # every rank reads S, writes S/p
    if op == "lastaxis":
        return 2 * p * S if algo == "gather" else p * S + S
    if op == "bcast":  # pull: p-1 ranks read S and write S; push: the root reads S once, p-1 writes of S
        return 2 * (p - 1) * S if algo == "direct" else p * S
    return 0.0


def bus_factor(op: str) -> float:
    if p == 1:
        return 0.0
    if op == "bcast":
        return 1.0
    return 2 * (p - 1) / p if op == "allreduce" else (p - 1) / p


# one symmetric arena per rank big enough for the largest op (2 x maxb)
arena_in = dev.empty(maxb // es + 64, dt)
arena_out = dev.empty(maxb // es + 64, dt)


def make(op: str, algo: str, S: int, mb: int):
    """(callable, checker) for one point; S in bytes."""
    n = S // es
    x, y = arena_in[:n], arena_out[:n]
    kw = {"max_blocks": mb} if mb else {}
    if op == "allreduce":
        x.fill_(rank + 1)
        want = p * (p + 1) / 2
        return (lambda: dev.allreduce(x, y, "SUM", algo, **kw)), (lambda: bool(torch.all(y == want).item()))
    if op == "allgather":
        xi = x[: n // p]
        xi.fill_(rank + 1)
        ref = torch.arange(1, p + 1, device=dev.device, dtype=dt).repeat_interleave(n // p)
        return (lambda: dev.allgather(xi, y[: n // p * p], algo, **kw)), (lambda: bool(torch.equal(y[: n // p * p], ref)))
    if op == "reduce_scatter":
        x.fill_(rank + 1)
        yo = y[: n // p]
        want = p * (p + 1) / 2
        return (lambda: dev.reduce_scatter(x[: n // p * p], yo, "SUM", algo, **kw)), (lambda: bool(torch.all(yo == want).item()))
    if op == "alltoall":
        blk = n // p
        x[: blk * p].view(p, blk).copy_((rank * p + torch.arange(p, device=dev.device, dtype=dt)).view(p, 1).expand(p, blk))
        ref = (torch.arange(p, device=dev.device, dtype=dt) * p + rank).view(p, 1).expand(p, blk).reshape(-1)
        return (lambda: dev.alltoall(x[: blk * p], y[: blk * p], algo, **kw)), (lambda: bool(torch.equal(y[: blk * p], ref)))
    if op == "lastaxis":
        # (rows, k) shards <-> (rows, p*k): k = 1024 elements per row shard
        k = 1024
        rows = max(1, n // (p * k))
        if algo == "gather":
            xi = arena_in[: rows * k]
            xi.fill_(rank + 1)
            yo = arena_out[: rows * k * p]
            ref = torch.arange(1, p + 1, device=dev.device, dtype=dt).repeat_interleave(k).repeat(rows)
            return (lambda: dev.allgather_lastaxis(xi, yo, rows, k * es)), (lambda: bool(torch.equal(yo, ref)))
        xi = arena_in[: rows * k * p]
        xi.fill_(rank + 1)
        yo = arena_out[: rows * k]
        want = p * (p + 1) / 2
        return (lambda: dev.reduce_scatter_lastaxis(xi, yo, rows, k)), (lambda: bool(torch.all(yo == want).item()))
    if op == "bcast":
        root = p - 1
        x.fill_(rank + 1)
        return (lambda: dev.bcast(x, root, algo)), (lambda: bool(torch.all(x == root + 1).item()))
    raise ValueError(op)


def time_point(fn, iters: int) -> float:
    fn()
    torch.cuda.synchronize()
    hc.Barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    return hc.allreduce(t, op=MPI.MAX)


lines = []
blocks = [int(b) for b in args.blocks.split(",")]
for op in ops:
    algos = DEFAULT_ALGOS[op]
    if args.algos:  # the requested algorithms this op has (lastaxis: gather / rscatter)
        valid = set(DEFAULT_ALGOS[op]) | {"rccl"} \
            | ({"pairwise"} if op == "alltoall" else set())
        algos = [a for a in args.algos.split(",") if a in valid] or DEFAULT_ALGOS[op]
    for algo in algos:
        for mb in blocks:
            S = args.min_bytes
            failed = False
            while S <= maxb and not failed:
                if op == "allreduce" and algo == "oneshot" and S > (64 << 20):
                    break
                if op == "allreduce" and algo == "ll" and S > dev.ll_max:
                    break
                if op == "allreduce" and algo == "reduce_bcast" and S > (256 << 20):
                    break
                Sx = S // (16 * p) * (16 * p)  # every rank's block 16-B aligned
                if Sx == 0:
                    S *= args.factor
                    continue
                ok = 1
                err = ""
                try:
                    fn, chk = make(op, algo, Sx, mb)
                    fn()
                    torch.cuda.synchronize()
                    dev.check()
                    ok = int(chk())
                except Exception as e:  # noqa: BLE001 - recorded in the output line
                    ok, err = 0, f"{type(e).__name__}: {e}"[:300]
                ok = hc.allreduce(ok, op=MPI.MIN)
                rec = {"op": op, "algo": algo, "blocks": mb or dev.max_blocks, "size": Sx, "ranks": p,
                       "shared_gpu": dev.shared_device, "dtype": args.dtype}
                if not ok:
                    rec["error"] = err or "wrong result"
                    failed = True
                    if err.startswith("RuntimeError: device collective timeout"):
                        dev.reset()
                else:
                    iters = args.iters or int(min(200, max(5, 4e8 / max(Sx, 1) / max(1, p))))
                    t = time_point(fn, iters)
                    hb = hbm_model(op, algo, Sx)
                    rec.update({"iters": iters, "us": round(t * 1e6, 2), "algbw_GBps": round(Sx / t / 1e9, 2),
                                "busbw_GBps": round(Sx / t / 1e9 * bus_factor(op), 2), "hbm_bytes": int(hb),
                                "hbm_GBps": round(hb / t / 1e9, 1), "hbm_frac": round(hb / t / HBM_CEIL, 3)})
                if rank == 0:
                    lines.append(rec)
                    print(json.dumps(rec), flush=True)
                S *= args.factor
dev.check()
if rank == 0 and args.out:
    with open(args.out, "w") as f:
        for r in lines:
            f.write(json.dumps(r) + "\n")
