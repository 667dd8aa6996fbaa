"""MoE-shaped all-to-all (BASELINE config: "pairwise all-to-all, 8xMI355X,
256 MiB/rank, nonblocking Isend/Irecv path").

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/alltoall_moe.py --mb 256
    scripts/mpirun -n 2 python benchmarks/alltoall_moe.py --mb 64      # ranks sharing one GPU

Algorithms: ``direct`` (hand-written kernel: every rank pulls its block from
all peers at once over xGMI), ``push`` (every rank writes its segments straight
into the peers' outputs, the reference myAlltoall pattern), ``pairwise`` (reference myAlltoall2 schedule on
RCCL send/recv rounds), ``rccl`` (ncclAllToAll, the library baseline).  Each is
checked for exactness, then timed (median of --iters).  Prints one JSON line.
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
ap.add_argument("--mb", type=int, default=256, help="send buffer per rank (MiB)")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--warmup", type=int, default=3)
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
dev = comm.dev
hc = comm.comm
n = (args.mb << 20) // 4 // p * p
x = dev.empty(n, torch.float32)
y = dev.empty(n, torch.float32)
blk = n // p
# element i of block j = rank*1e6 + j*1e3 + (i % 997): checkable on the receiver
ar = torch.arange(blk, device=dev.device, dtype=torch.float32) % 997
for j in range(p):
    x[j * blk:(j + 1) * blk] = rank * 1e6 + j * 1e3 + ar
algos = ["direct", "push"] + ([] if dev.shared_device else ["pairwise", "rccl"])
res = {}
for algo in algos:
    try:
        dev.alltoall(x, y, algo)
        torch.cuda.synchronize()
        dev.check()
        ok = all(torch.equal(y[j * blk:(j + 1) * blk], j * 1e6 + rank * 1e3 + ar) for j in range(p))
    except Exception as e:  # noqa: BLE001
        ok = False
        if rank == 0:
            print(f"# {algo}: {e}", file=sys.stderr)
    if not hc.allreduce(int(ok), op=MPI.MIN):
        res[algo] = None
        continue
    for _ in range(args.warmup):
        dev.alltoall(x, y, algo)
    ts = []
    for _ in range(args.iters):
        torch.cuda.synchronize()
        hc.Barrier()
        t0 = time.perf_counter()
        dev.alltoall(x, y, algo)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res[algo] = hc.allreduce(statistics.median(ts), op=MPI.MAX)
if rank == 0:
    nbytes = n * 4
    out = {"bench": "alltoall_moe", "ranks": p, "bytes_per_rank": nbytes, "shared_gpu": dev.shared_device,
           "hbm_bytes_all_ranks": 2 * p * nbytes,
           "results": {a: (None if t is None else {"ms": round(t * 1e3, 4),
                                                   "algbw_GBps": round(nbytes / t / 1e9, 2),
                                                   "busbw_GBps": round(nbytes / t / 1e9 * (p - 1) / p, 2)})
                       for a, t in res.items()}}
    print(json.dumps(out), flush=True)
