"""Demo / benchmark CLI with the reference's test cases (reference mpi-test.py:1-241).

    scripts/mpirun -n 8 python mpi-test.py --test_case myallreduce
    scripts/mpirun -n 8 python mpi-test.py --test_case myalltoall --device cuda --size 1048576

Cases: allreduce, allgather, reduce_scatter, split, alltoall, myallreduce,
myalltoall (same output lines as the reference), plus:

* ``--device cpu|cuda``: host buffers go through the shared-memory plane; CUDA buffers go through the
  device plane.  Under ``cuda`` the "library" baseline is RCCL when it can be used (one rank per GPU),
  and the framework's default algorithm otherwise.
* ``--size/--dtype/--algo/--runs/--seed``.

Deliberate differences from the reference:
* allgather / reduce_scatter are sized by the comm size, not hard-coded for 8 ranks;
* ``--test_case allreduce`` no longer also prints "This is rank N." (an if/elif slip at mpi-test.py:40);
* inputs are seeded (``--seed``) so runs are reproducible.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from collective_communication_mpi_amd import MPI  # noqa: E402
from mpi_wrapper import Communicator  # noqa: E402

CASES = ["allreduce", "allgather", "reduce_scatter", "split", "alltoall", "myallreduce", "myalltoall"]
parser = argparse.ArgumentParser()
parser.add_argument("--test_case", type=str, default="", choices=CASES + [""],
                    help="MPI names for different toy examples")
parser.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
parser.add_argument("--size", type=int, default=100, help="elements for myallreduce (reference: 100)")
parser.add_argument("--dtype", default="int64")
parser.add_argument("--algo", default="", help="myAllreduce/myAlltoall algorithm (default: reference algorithm)")
parser.add_argument("--runs", "--iters", type=int, default=100, help="timed runs (reference: 100)")
parser.add_argument("--warmup", type=int, default=0, help="untimed runs before the timed ones")
parser.add_argument("--seed", type=int, default=0)


class Buffers:
    """Allocates host or device buffers for the demo."""

    def __init__(self, device, comm):
        self.device = device
        self.comm = comm
        if device == "cuda":
            import torch

            self.torch = torch
            local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
            torch.cuda.set_device(local % torch.cuda.device_count())

    def put(self, a):
        if self.device == "cpu":
            return a
        return self.torch.from_numpy(np.ascontiguousarray(a)).cuda()

    def empty(self, n, dtype):
        if self.device == "cpu":
            return np.empty(n, dtype=dtype)
        return self.torch.empty(n, dtype=getattr(self.torch, np.dtype(dtype).name), device="cuda")

    def get(self, x):
        if self.device == "cpu":
            return x
        self.torch.cuda.synchronize()
        return x.cpu().numpy()

    def sync(self):
        if self.device == "cuda":
            self.torch.cuda.synchronize()


def library_algo(comm, device):
    """'library' baseline: MPI built-ins on CPU, RCCL on GPU when usable."""
    if device == "cpu":
        return "auto"
    return "auto" if comm.dev.shared_device else "rccl"


def timed_compare(comm, bufs, args, make_input, library, mine, label, lib_label):
    rank = comm.Get_rank()
    rng = np.random.default_rng(args.seed + rank)
    lib_times, my_times = [], []
    all_ok = True
    for _ in range(args.warmup):  # untimed: first-touch, RCCL/IPC setup, kernel loads
        src, n, dtype = make_input(rng)
        library(src, bufs.empty(n, dtype))
        mine(src, bufs.empty(n, dtype))
        bufs.sync()
    comm.Barrier()
    for run in range(args.runs):
        src, n, dtype = make_input(rng)
        a = bufs.empty(n, dtype)
        b = bufs.empty(n, dtype)
        bufs.sync()
        comm.Barrier()
        t = MPI.Wtime()
        library(src, a)
        bufs.sync()
        comm.Barrier()
        lib_times.append(MPI.Wtime() - t)
        comm.Barrier()
        t = MPI.Wtime()
        mine(src, b)
        bufs.sync()
        comm.Barrier()
        my_times.append(MPI.Wtime() - t)
        ra, rb = bufs.get(a), bufs.get(b)
        if not np.array_equal(ra, rb):
            all_ok = False
            print("Rank {}: Run {}: ERROR: {} result does not match {}".format(rank, run, label, lib_label))
            if rank == 0:
                print("{} result:   ".format(lib_label), ra)
                print("{} result: ".format(label), rb)
        elif rank == 0:
            print("Run {}: Correct results.".format(run))
    if rank == 0:
        print("\nSummary over {} runs:".format(args.runs))
        print("All runs produced correct results." if all_ok else "Some runs produced incorrect results!")
        print("Average {} time: {:.6f} seconds".format(lib_label, sum(lib_times) / args.runs))
        print("Average {} time:   {:.6f} seconds".format(label, sum(my_times) / args.runs))
    return all_ok


def main():
    args = parser.parse_args()
    comm = Communicator(MPI.COMM_WORLD)
    nprocs = comm.Get_size()
    rank = comm.Get_rank()
    bufs = Buffers(args.device, comm)
    rng = np.random.default_rng(args.seed + rank)
    case = args.test_case

    if case == "allreduce":
        r = rng.integers(0, 100, 100)
        rr = bufs.empty(100, np.int64)
        print("Rank " + str(rank) + ": " + str(r))
        comm.Barrier()
        comm.Allreduce(bufs.put(r), rr, op=MPI.MIN)
        if rank == 0:
            print("Allreduce: " + str(bufs.get(rr)))
    elif case == "myallreduce":
        dtype = np.dtype(args.dtype)
        algo = args.algo or "reduce_bcast"
        lib = library_algo(comm, args.device)

        def make(rng_):
            return bufs.put(rng_.integers(0, 100, args.size).astype(dtype)), args.size, dtype

        ok = timed_compare(comm, bufs, args, make,
                           lambda s, d: comm.Allreduce(s, d, op=MPI.MIN, **({"algo": lib} if args.device == "cuda" else {})),
                           lambda s, d: comm.myAllreduce(s, d, op=MPI.MIN, algo=algo),
                           "myAllreduce", "MPI.Allreduce")
        sys.exit(0 if ok else 1)
    elif case == "allgather":
        r = rng.integers(0, 100, 2)
        rr = bufs.empty(2 * nprocs, np.int64)
        print("Rank " + str(rank) + ": " + str(r))
        comm.Barrier()
        comm.Allgather(bufs.put(r), rr)
        if rank == 0:
            print("Allgather: " + str(bufs.get(rr)))
    elif case == "reduce_scatter":
        r = rng.integers(0, 100, 2 * nprocs)
        rr = bufs.empty(2, np.int64)
        print("Rank " + str(rank) + ": " + str(r))
        comm.Barrier()
        comm.Reduce_scatter(bufs.put(r), rr, op=MPI.MIN)
        print("Rank " + str(rank) + " After Reduce_scatter: " + str(bufs.get(rr)))
    elif case == "split":
        r = rng.integers(0, 100, 10)
        rr = bufs.empty(10, np.int64)
        print("Rank " + str(rank) + ": " + str(r))
        group_comm = comm.Split(key=rank, color=rank % 4)
        group_comm.Barrier()
        group_comm.Allreduce(bufs.put(r), rr, op=MPI.MIN)
        print("Rank " + str(rank) + " After split and Allreduce: " + str(bufs.get(rr)))
    elif case == "alltoall":
        send = np.array([rank * 100 + i for i in range(nprocs)], dtype=np.int64)
        recv = bufs.empty(nprocs, np.int64)
        print("Rank " + str(rank) + " sending: " + str(send))
        comm.Barrier()
        comm.Alltoall(bufs.put(send), recv)
        print("Rank " + str(rank) + " received: " + str(bufs.get(recv)))
    elif case == "myalltoall":
        n = max(nprocs, args.size // nprocs * nprocs) if args.size != 100 else nprocs
        algo = args.algo or "direct"
        lib = library_algo(comm, args.device)

        def make(rng_):
            # element i of segment j is rank*100 + j (reference: send_data[i] = rank*100 + i, one per rank)
            return bufs.put(rank * 100 + np.arange(n, dtype=np.int64) // max(1, n // nprocs)), n, np.int64

        ok = timed_compare(comm, bufs, args, make,
                           lambda s, d: comm.Alltoall(s, d, **({"algo": lib} if args.device == "cuda" else {})),
                           lambda s, d: comm.myAlltoall(s, d, **({"algo": algo} if args.device == "cuda" else {})),
                           "myAlltoall", "MPI.Alltoall")
        sys.exit(0 if ok else 1)
    else:
        print(f"This is rank {rank}.")


if __name__ == "__main__":
    main()
