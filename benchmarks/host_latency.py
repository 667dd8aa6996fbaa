"""Host-plane (CPU) latency benchmark: BASELINE config 1, "myAllreduce 8-proc CPU
on a 1k-float32 buffer", plus the primitives under it.

    scripts/mpirun -n 8 python benchmarks/host_latency.py [--iters 2000]

Per op: median and p10 over ``--reps`` repetitions of ``--iters`` back-to-back
calls (no barrier inside the timed loop; one barrier before each repetition).
Ops: one-way Send/Recv latency between ranks 0 and 1 (ping-pong / 2), Barrier,
Allreduce (library path), myAllreduce (reference reduce->bcast schedule, plus
ring and rhd), Alltoall and myAlltoall/myAlltoall2, the non-blocking
Iallreduce/Ialltoall/Ibarrier (+ Wait), all on the float32 buffer
of ``--count`` elements (alltoall: ``--count`` per rank in total).  Rank 0
prints one JSON line.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--count", type=int, default=1024)
ap.add_argument("--iters", type=int, default=2000)
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
comm = MPI.COMM_WORLD
C = Communicator(comm)
rank, p = comm.Get_rank(), comm.Get_size()
x = np.random.default_rng(rank).standard_normal(args.count).astype(np.float32)
y = np.empty_like(x)
n_a2a = args.count // p * p
xa, ya = x[:n_a2a].copy(), np.empty(n_a2a, np.float32)


def timeit(fn, iters=args.iters):
    ts = []
    for _ in range(args.reps):
        comm.Barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        ts.append((time.perf_counter() - t0) / iters)
    worst = comm.allgather(statistics.median(ts))
    return {"median_us": round(max(worst) * 1e6, 3), "p10_us": round(sorted(ts)[len(ts) // 10] * 1e6, 3)}


res = {}
if p >= 2:
    def pingpong():
        if rank == 0:
            comm.Send(x, dest=1)
            comm.Recv(y, source=1)
        elif rank == 1:
            comm.Recv(y, source=0)
            comm.Send(x, dest=0)
    r = timeit(pingpong)
    res["sendrecv_one_way"] = {k: round(v / 2, 3) for k, v in r.items()}
res["barrier"] = timeit(comm.Barrier)
res["Allreduce"] = timeit(lambda: C.Allreduce(x, y, op=MPI.SUM))
for algo in ("reduce_bcast", "ring", "rhd"):
    res[f"myAllreduce_{algo}"] = timeit(lambda: C.myAllreduce(x, y, op=MPI.SUM, algo=algo), args.iters // 4)
res["Alltoall"] = timeit(lambda: C.Alltoall(xa, ya))
res["myAlltoall"] = timeit(lambda: C.myAlltoall(xa, ya), args.iters // 4)
res["myAlltoall2"] = timeit(lambda: C.myAlltoall2(xa, ya), args.iters // 4)
# MPI-3 non-blocking collectives (csrc/host/nbcoll.cpp), started and waited at once
res["Iallreduce+Wait"] = timeit(lambda: comm.Iallreduce(x, y, MPI.SUM).Wait(), args.iters // 4)
res["Ialltoall+Wait"] = timeit(lambda: comm.Ialltoall(xa, ya).Wait(), args.iters // 4)
res["Ibarrier+Wait"] = timeit(lambda: comm.Ibarrier().Wait(), args.iters // 4)
if rank == 0:
    print(json.dumps({"bench": "host_latency", "ranks": p, "count": args.count, "dtype": "float32",
                      "cpus": os.cpu_count(), "results_us": res}), flush=True)
