"""MoE-shaped all-to-all (BASELINE config: "pairwise all-to-all, 8xMI355X,
256 MiB/rank, nonblocking Isend/Irecv path").

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/alltoall_moe.py --mb 256
    scripts/mpirun -n 2 python benchmarks/alltoall_moe.py --mb 64      # ranks sharing one GPU

Algorithms: ``direct`` (hand-written kernel: every rank pulls its block from
all peers at once over xGMI), ``push`` (every rank writes its segments straight
into the peers' outputs, the reference myAlltoall pattern), ``pairwise`` (reference myAlltoall2 schedule on
RCCL send/recv rounds), ``rccl`` (ncclAllToAll, the library baseline).  Each is
checked for exactness, then timed (median of --iters).  Also the ragged
all-to-all (``alltoallv``: equal counts, and skewed MoE-like counts whose
correctness the device tests cover).  Prints one JSON line.
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
# ragged (MoE routing with imbalanced experts): alltoallv with counts drawn from a
# skewed distribution around the uniform block (same total per rank on average);
# "uniform" = alltoallv with equal counts, to compare against the push all-to-all
import random  # noqa: E402

rg = random.Random(7)
W = [[rg.choice([0.25, 0.5, 1.0, 1.0, 1.5, 2.0]) for _ in range(p)] for _ in range(p)]
Cr = [[int(blk * w / 2) // 4 * 4 for w in row] for row in W]  # 16-B segments (fp32 x 4)
for name, C in (("alltoallv_uniform", [[blk] * p for _ in range(p)]), ("alltoallv_ragged", Cr)):
    sc, rc = C[rank], [C[i][rank] for i in range(p)]
    xs, ys = x[:sum(sc)], y[:max(1, sum(rc))]
    try:
        dev.alltoallv(xs, sc, ys, rc)
        torch.cuda.synchronize()
        dev.check()
        o, ok = 0, True
        for i in range(p):  # from rank i: its send elements [sum(C[i][:rank]), + rc[i])
            g = torch.arange(sum(C[i][:rank]), sum(C[i][:rank]) + rc[i], device=dev.device)
            want = i * 1e6 + (g // blk).float() * 1e3 + (g % blk % 997).float()
            ok = ok and torch.equal(ys[o:o + rc[i]], want)
            o += rc[i]
    except Exception as e:  # noqa: BLE001
        ok = False
        if rank == 0:
            print(f"# {name}: {e}", file=sys.stderr)
    if not hc.allreduce(int(ok), op=MPI.MIN):
        res[name] = None
        continue
    for _ in range(args.warmup):
        dev.alltoallv(xs, sc, ys, rc)
    ts = []
    for _ in range(args.iters):
        torch.cuda.synchronize()
        hc.Barrier()
        t0 = time.perf_counter()
        dev.alltoallv(xs, sc, ys, rc)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res[name] = hc.allreduce(statistics.median(ts), op=MPI.MAX)
    res[name + "_max_send_bytes"] = max(sum(r) for r in C) * 4
# the ragged counts kept on the device (no host exchange): kernel-side count exchange
C = Cr
sc_dev = torch.tensor(C[rank], dtype=torch.int64, device=dev.device)
rc_dev = torch.empty(p, dtype=torch.int64, device=dev.device)
xs = x[:sum(C[rank])]
try:
    dev.alltoallv(xs, sc_dev, y, rc_dev)
    torch.cuda.synchronize()
    dev.check()
    ok = rc_dev.tolist() == [C[i][rank] for i in range(p)]
except Exception as e:  # noqa: BLE001
    ok = False
    if rank == 0:
        print(f"# alltoallv_devcounts: {e}", file=sys.stderr)
if hc.allreduce(int(ok), op=MPI.MIN):
    for _ in range(args.warmup):
        dev.alltoallv(xs, sc_dev, y, rc_dev)
    ts = []
    for _ in range(args.iters):
        torch.cuda.synchronize()
        hc.Barrier()
        t0 = time.perf_counter()
        dev.alltoallv(xs, sc_dev, y, rc_dev)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res["alltoallv_ragged_devcounts"] = hc.allreduce(statistics.median(ts), op=MPI.MAX)
else:
    res["alltoallv_ragged_devcounts"] = None
if rank == 0:
    nbytes = n * 4
    out = {"bench": "alltoall_moe", "ranks": p, "bytes_per_rank": nbytes, "shared_gpu": dev.shared_device,
           "hbm_bytes_all_ranks": 2 * p * nbytes,
           "results": {a: (None if t is None else t if a.endswith("_bytes") else
                               {"ms": round(t * 1e3, 4), "algbw_GBps": round(nbytes / t / 1e9, 2),
                                "busbw_GBps": round(nbytes / t / 1e9 * (p - 1) / p, 2)})
                       for a, t in res.items()}}
    print(json.dumps(out), flush=True)
