"""Non-blocking collectives of the host plane (csrc/host/nbcoll.cpp) and the
Communicator façade, checked against the blocking collectives / NumPy on every
rank.  Run under scripts/mpirun at any rank count."""
import faulthandler
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

if os.environ.get("NB_DUMP"):  # debugging a hang: dump every stack after NB_DUMP seconds
    faulthandler.dump_traceback_later(int(os.environ["NB_DUMP"]), exit=True)

comm = MPI.COMM_WORLD
rank, p = comm.Get_rank(), comm.Get_size()
fails = []


def check(ok, what):
    if not ok:
        fails.append(what)


def data(r, n, dt, salt=0):
    g = np.random.default_rng(1000 * salt + 17 * r + n)
    if np.dtype(dt).kind == "f":
        return (g.integers(-8, 8, n)).astype(dt)  # integral values: sums are exact in any order
    return g.integers(-50, 50, n).astype(dt)


ops = {"SUM": (MPI.SUM, np.add), "PROD": (MPI.PROD, np.multiply), "MIN": (MPI.MIN, np.minimum),
       "MAX": (MPI.MAX, np.maximum)}

# ---- Iallreduce: small (all-pairs) and large (ring) schedules, every op, several dtypes
for n in (0, 1, p - 1 if p > 1 else 1, 37, 4096, 70001):
    for dt in ("float32", "int64", "float64", "int32"):
        for name, (op, f) in ops.items():
            if name == "PROD" and n > 64:
                continue
            x = data(rank, n, dt)
            want = data(0, n, dt)
            for r in range(1, p):
                want = f(want, data(r, n, dt))
            y = np.full(n, -1, dt)
            req = comm.Iallreduce(x, y, op)
            req.Wait()
            check(np.array_equal(y, want), f"Iallreduce n={n} {dt} {name}")
            z = x.copy()
            comm.Iallreduce(MPI.IN_PLACE, z, op).Wait()
            check(np.array_equal(z, want), f"Iallreduce in-place n={n} {dt} {name}")

# ---- Iallgather / Ialltoall / Ireduce_scatter_block / Ibcast
for blk in (0, 1, 5, 3000, 40000):
    x = data(rank, blk, "float32", 1)
    y = np.zeros(blk * p, np.float32)
    comm.Iallgather(x, y).Wait()
    check(np.array_equal(y, np.concatenate([data(r, blk, "float32", 1) for r in range(p)])), f"Iallgather blk={blk}")
    z = np.zeros(blk * p, np.float32)
    z[rank * blk:(rank + 1) * blk] = x
    comm.Iallgather(MPI.IN_PLACE, z).Wait()
    check(np.array_equal(z, y), f"Iallgather in-place blk={blk}")

    a = (np.arange(p * blk, dtype=np.int64) + 1000000 * rank)
    b = np.zeros_like(a)
    comm.Ialltoall(a, b).Wait()
    want = np.concatenate([np.arange(rank * blk, (rank + 1) * blk, dtype=np.int64) + 1000000 * r for r in range(p)])
    check(np.array_equal(b, want), f"Ialltoall blk={blk}")
    comm.Ialltoall(MPI.IN_PLACE, a).Wait()
    check(np.array_equal(a, want), f"Ialltoall in-place blk={blk}")

    s = data(rank, blk * p, "int32", 2)
    rs = np.zeros(blk, np.int32)
    comm.Ireduce_scatter_block(s, rs, MPI.SUM).Wait()
    tot = sum(data(r, blk * p, "int32", 2).astype(np.int64) for r in range(p)).astype(np.int32)
    check(np.array_equal(rs, tot[rank * blk:(rank + 1) * blk]), f"Ireduce_scatter_block blk={blk}")
    ip = s.copy()
    comm.Ireduce_scatter_block(MPI.IN_PLACE, ip, MPI.MAX).Wait()
    mx = np.maximum.reduce([data(r, blk * p, "int32", 2) for r in range(p)]) if blk else np.zeros(0, np.int32)
    check(np.array_equal(ip[:blk], mx[rank * blk:(rank + 1) * blk]), f"Ireduce_scatter_block in-place blk={blk}")

    for root in {0, p - 1, p // 2}:
        bb = data(root, blk * 3, "float64", 3) if rank == root else np.zeros(blk * 3)
        comm.Ibcast(bb, root).Wait()
        check(np.array_equal(bb, data(root, blk * 3, "float64", 3)), f"Ibcast blk={blk} root={root}")

# ---- Ibarrier: nobody leaves before the last rank arrived
t_arrive = np.zeros(1)
if rank == p - 1:
    time.sleep(0.2)
t_arrive[0] = time.time()
req = comm.Ibarrier()
while not req.Test():
    pass
t_leave = time.time()
last = np.zeros(1)
comm.Allreduce(t_arrive, last, MPI.MAX)
check(t_leave >= last[0] - 1e-3, "Ibarrier released early")

# ---- many collectives in flight at once, completed in reverse order, with user
# P2P traffic on ANY_TAG in between (internal tags must not match it)
n = 50000
xs = [data(rank, n, "float32", 10 + i) for i in range(6)]
ys = [np.zeros(n, np.float32) for _ in range(6)]
reqs = [comm.Iallreduce(xs[i], ys[i], MPI.SUM) for i in range(4)]
ag_out = np.zeros(p * 7, np.float64)
reqs.append(comm.Iallgather(np.full(7, float(rank)), ag_out))
reqs.append(comm.Ibarrier())
if p > 1:
    tok = np.array([rank], np.int64)
    got = np.zeros(1, np.int64)
    st = MPI.Status()
    rq = comm.Irecv(got, source=MPI.ANY_SOURCE, tag=MPI.ANY_TAG)
    comm.Send(tok, dest=(rank + 1) % p, tag=7)
    rq.Wait(st)
    check(got[0] == (rank - 1) % p and st.Get_tag() == 7, "user P2P mixed with collectives")
for r in reversed(reqs):
    r.Wait()
for i in range(4):
    check(np.array_equal(ys[i], sum(data(r, n, "float32", 10 + i) for r in range(p))), f"in-flight Iallreduce {i}")
check(np.array_equal(ag_out, np.repeat(np.arange(p, dtype=np.float64), 7)), "in-flight Iallgather")
check(comm._hc.nb_active == 0, "collectives left active")

# ---- a rank blocked in an unrelated receive still forwards ring rounds: rank 0
# waits for a message that its right neighbour sends only after ITS all-reduce
# completed, so that all-reduce must progress inside rank 0's blocking Recv
if p > 1:
    big = data(rank, 200000, "float32", 20)
    out = np.zeros_like(big)
    req = comm.Iallreduce(big, out, MPI.SUM)
    if rank == 0:
        m = np.zeros(1)
        comm.Recv(m, source=1, tag=99)
        req.Wait()
    else:
        req.Wait()
        if rank == 1:
            comm.Send(np.ones(1), dest=0, tag=99)
    check(np.array_equal(out, sum(data(r, 200000, "float32", 20) for r in range(p))), "progress inside Recv")

# ---- Waitall over host P2P + collective requests
if p > 1:
    rb = np.zeros(3, np.int32)
    a = comm.Irecv(rb, source=(rank - 1) % p, tag=3)
    b = comm.Isend(np.full(3, rank, np.int32), dest=(rank + 1) % p, tag=3)
    ar = np.zeros(5, np.int32)
    c = comm.Iallreduce(np.full(5, rank, np.int32), ar, MPI.SUM)
    MPI.Request.Waitall([a, b, c])
    check(np.array_equal(rb, np.full(3, (rank - 1) % p)) and np.array_equal(ar, np.full(5, p * (p - 1) // 2)),
          "Waitall mixed")

# ---- a request dropped unwaited: the communicator keeps its buffers alive and later
# waits keep progressing it to completion (no use-after-free, nothing left active)
import gc  # noqa: E402

comm.Iallreduce(np.arange(100000, dtype=np.float64) * (rank + 1), np.zeros(100000), MPI.SUM)
gc.collect()
junk = [np.full(100000, 7.0) for _ in range(8)]  # reuse freed memory if it had been freed
for _ in range(1000):
    comm.Ibarrier().Wait()
    if comm.allreduce(comm._hc.nb_active, op=MPI.MAX) == 0:  # collective exit decision
        break
check(comm._hc.nb_active == 0, "dropped request never completed")
del junk

# ---- Communicator façade: same results and byte accounting as the blocking calls
cm = Communicator(comm)
x = data(rank, 1000, "float32", 30)
y1, y2 = np.zeros_like(x), np.zeros_like(x)
cm.Allreduce(x, y1, MPI.SUM)
b0 = cm.total_bytes_transferred
cm.Iallreduce(x, y2, MPI.SUM).Wait()
check(np.array_equal(y1, y2) and cm.total_bytes_transferred == 2 * b0, "Communicator.Iallreduce")
a = np.arange(p * 4, dtype=np.float32) + rank
o1, o2 = np.zeros_like(a), np.zeros_like(a)
cm.Alltoall(a, o1)
cm.Ialltoall(a, o2).Wait()
check(np.array_equal(o1, o2), "Communicator.Ialltoall")
g1, g2 = np.zeros(p * 4, np.float32), np.zeros(p * 4, np.float32)
cm.Allgather(a[:4], g1)
cm.Iallgather(a[:4], g2).Wait()
check(np.array_equal(g1, g2), "Communicator.Iallgather")
r1, r2 = np.zeros(4, np.float32), np.zeros(4, np.float32)
cm.Reduce_scatter(a, r1, MPI.SUM)
cm.Ireduce_scatter(a, r2, MPI.SUM).Wait()
check(np.array_equal(r1, r2), "Communicator.Ireduce_scatter")
cm.Ibarrier().Wait()
# Alltoallv on the host plane (ragged counts, packed in rank order)
C = [[(3 * i + j) % 4 for j in range(p)] for i in range(p)]
src = np.concatenate([np.full(C[rank][j], 100 * rank + j, np.int32) for j in range(p)] or [np.zeros(0, np.int32)])
dst = np.full(max(1, sum(C[i][rank] for i in range(p))), -1, np.int32)
b0 = cm.total_bytes_transferred
cm.Alltoallv(src, C[rank], dst, [C[i][rank] for i in range(p)])
want = np.concatenate([np.full(C[i][rank], 100 * i + rank, np.int32) for i in range(p)])
check(np.array_equal(dst[:want.size], want), "Communicator.Alltoallv (host)")
check(cm.total_bytes_transferred - b0 == 4 * (sum(C[rank]) - C[rank][rank] + sum(C[i][rank] for i in range(p)) - C[rank][rank]),
      "Alltoallv accounting")

bad = comm.allgather(fails)
if rank == 0:
    allf = [f"rank {r}: {f}" for r, fl in enumerate(bad) for f in fl]
    if allf:
        print("FAILURES:\n" + "\n".join(allf[:40]))
        sys.exit(1)
    print(f"nonblocking collectives OK ({p} ranks)")
