"""Collective sweep: time vs message size for every device algorithm.

    scripts/mpirun -n 4 python benchmarks/sweep.py --op allreduce --max-mb 256
    torchrun --nproc-per-node 8 benchmarks/sweep.py --op all

Prints one JSON line per (op, algo, bytes) on rank 0 with time (us, median of
--iters after --warmup), algbw and busbw (NCCL-tests conventions:
all-reduce busbw = algbw * 2(p-1)/p; all-gather / reduce-scatter / all-to-all
busbw = algbw * (p-1)/p).  With several ranks on ONE GPU the numbers measure
protocol latency + HBM traffic, not xGMI.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--op", default="allreduce", help="allreduce|allgather|reduce_scatter|alltoall|all")
ap.add_argument("--algos", default="")
ap.add_argument("--min-bytes", type=int, default=1024)
ap.add_argument("--max-mb", type=int, default=64)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
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
big_in = dev.empty(maxb * max(1, p) // es, dt)
big_out = dev.empty(maxb * max(1, p) // es, dt)
big_in.fill_(1)
ops = ["allreduce", "allgather", "reduce_scatter", "alltoall"] if args.op == "all" else [args.op]
default_algos = {
    "allreduce": ["oneshot", "twoshot", "reduce_bcast"] + (["rccl", "ring"] if not dev.shared_device else []),
    "allgather": ["direct"] + (["rccl"] if not dev.shared_device else []),
    "reduce_scatter": ["direct"] + (["rccl"] if not dev.shared_device else []),
    "alltoall": ["direct"] + (["rccl", "pairwise"] if not dev.shared_device else []),
}
lines = []
for op in ops:
    algos = args.algos.split(",") if args.algos else default_algos[op]
    b = args.min_bytes
    while b <= maxb:
        n = max(1, b // es)
        for algo in algos:
            if op == "allreduce" and algo == "oneshot" and b > (64 << 20):
                continue
            if op == "allreduce":
                fn = lambda: dev.allreduce(big_in[:n], big_out[:n], "SUM", algo)  # noqa: E731
                factor = 2 * (p - 1) / p if p > 1 else 0
            elif op == "allgather":
                fn = lambda: dev.allgather(big_in[:n], big_out[:n * p], algo)  # noqa: E731
                factor = (p - 1) / p
            elif op == "reduce_scatter":
                fn = lambda: dev.reduce_scatter(big_in[:n * p], big_out[:n], "SUM", algo)  # noqa: E731
                factor = (p - 1) / p
            else:
                nn = max(p, n // p * p)
                fn = lambda: dev.alltoall(big_in[:nn], big_out[:nn], algo)  # noqa: E731
                factor = (p - 1) / p
            try:
                for _ in range(args.warmup):
                    fn()
                torch.cuda.synchronize()
                ts = []
                for _ in range(args.iters):
                    hc.Barrier()
                    t0 = time.perf_counter()
                    fn()
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                t = hc.allreduce(statistics.median(ts), op=MPI.MAX)
            except Exception as e:  # noqa: BLE001
                t = None
                if rank == 0:
                    print(f"# {op}/{algo} @ {b}: {e}", file=sys.stderr)
            if rank == 0 and t:
                rec = {"op": op, "algo": algo, "bytes": n * es, "ranks": p, "shared_gpu": dev.shared_device,
                       "us": round(t * 1e6, 2), "algbw_GBps": round(n * es / t / 1e9, 3),
                       "busbw_GBps": round(n * es / t / 1e9 * factor, 3)}
                lines.append(rec)
                print(json.dumps(rec), flush=True)
        b *= 4
dev.check()
if rank == 0 and args.out:
    with open(args.out, "w") as f:
        for r in lines:
            f.write(json.dumps(r) + "\n")
