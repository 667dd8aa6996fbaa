"""Where the host-plane ranks run: each rank's allowed CPU set, the L3 domain of its CPU, and
the CPU it is on before / after each of a few hundred reduce->bcast calls (fresh arrays),
to see whether ranks share an L3 and whether the scheduler migrates them."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

libc = ctypes.CDLL(None)
world = MPI.COMM_WORLD
comm = Communicator(world)
rank, p = comm.Get_rank(), comm.Get_size()
rng = np.random.default_rng(rank)


def l3_of(cpu):
    try:
        with open(f"/sys/devices/system/cpu/cpu{cpu}/cache/index3/shared_cpu_list") as f:
            return f.read().strip()
    except OSError:
        return "?"


cpus = []
for _ in range(300):
    s = rng.standard_normal(1024).astype(np.float32)
    d = np.empty(1024, np.float32)
    comm.Barrier()
    c0 = libc.sched_getcpu()
    comm.myAllreduce(s, d, op=MPI.MIN)
    cpus.append((c0, libc.sched_getcpu()))
aff = sorted(os.sched_getaffinity(0))
info = {"rank": rank, "n_allowed": len(aff), "allowed_head": aff[:24], "distinct_cpus": len(set(c for pr in cpus for c in pr)),
        "first_cpu": cpus[0][0], "last_cpu": cpus[-1][1], "l3": l3_of(cpus[-1][1]),
        "migrations_in_call": sum(1 for a, b in cpus if a != b)}
allinfo = world.gather(info, root=0)
if rank == 0:
    for i in allinfo:
        print(json.dumps(i), flush=True)
