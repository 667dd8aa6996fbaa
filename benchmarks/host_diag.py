"""Host-plane all-reduce latency under the reference's per-run timing (Barrier, Wtime, call,
Barrier, Wtime; mpi-test.py:59-72), split into the call alone per rank and the trailing
barrier, for the library Allreduce and each hand-written myAllreduce schedule, with fresh or
reused buffers per run.  Rank 0 prints one JSON line per case (max over ranks of the mean)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

world = MPI.COMM_WORLD
comm = Communicator(world)
rank, p = comm.Get_rank(), comm.Get_size()
rng = np.random.default_rng(rank)
n = int(os.environ.get("HD_COUNT", "1024"))
runs = int(os.environ.get("HD_RUNS", "200"))


fresh_ranks = os.environ.get("HD_FRESH_RANKS")  # e.g. "0" or "1-7": only these ranks take fresh arrays
if fresh_ranks:
    lo, _, hi = fresh_ranks.partition("-")
    mine = int(lo) <= rank <= int(hi or lo)
else:
    mine = True


def run(name, fn, fresh):
    fresh = fresh if mine else False
    call, total = [], []
    s = rng.standard_normal(n).astype(np.float32)
    d = np.empty(n, np.float32)
    for _ in range(runs):
        if fresh in (True, "touched", "src"):
            s = rng.standard_normal(n).astype(np.float32)
        if fresh in (True, "touched", "dst"):
            d = np.empty(n, np.float32)
            if fresh == "touched":
                d.fill(0)
        comm.Barrier()
        t0 = MPI.Wtime()
        fn(s, d)
        t1 = MPI.Wtime()
        comm.Barrier()
        t2 = MPI.Wtime()
        call.append(t1 - t0)
        total.append(t2 - t0)
    per_rank_call = world.allgather(round(statistics.mean(call) * 1e6, 2))
    tot = max(world.allgather(statistics.mean(total)))
    if rank == 0:
        print(json.dumps({"case": name, "fresh": fresh, "avg_us": round(tot * 1e6, 2), "call_us_per_rank": per_rank_call}),
              flush=True)


cases = os.environ.get("HD_FRESH", "True,touched,False").split(",")
algos = os.environ.get("HD_ALGOS", "reduce_bcast,ring,rhd").split(",")
for fresh in [{"True": True, "False": False}.get(c, c) for c in cases]:
    run("Allreduce", lambda s, d: comm.Allreduce(s, d, op=MPI.MIN), fresh)
    for algo in algos:
        run(f"myAllreduce_{algo}", lambda s, d, a=algo: comm.myAllreduce(s, d, op=MPI.MIN, algo=a), fresh)
    run("Sendrecv_ring", lambda s, d: comm.comm.Sendrecv(s, dest=(rank + 1) % p, recvbuf=d, source=(rank - 1) % p), fresh)
    run("Barrier", lambda s, d: None, fresh)
