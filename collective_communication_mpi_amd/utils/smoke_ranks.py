"""Multi-rank smoke check of the hand-written device collectives (``__graft_entry__.smoke``).

    python -m collective_communication_mpi_amd.launch -n 2 --timeout 120 \
        python -m collective_communication_mpi_amd.utils.smoke_ranks

Every rank holds ``rank + 1`` in a 4 MiB fp32 and a bf16 buffer; each all-reduce algorithm
(two-shot, fan-out) must return ``p (p + 1) / 2`` everywhere, exactly.  With a single
process, an all-reduce is only a copy.  This check runs p >= 2 ranks of the real protocol:
IPC-mapped peers, signal flags and the reduction kernels.  On one GPU the ranks share it.
Rank 0 prints ``multi-rank smoke OK``.
"""
import os
import sys


def main() -> int:
    import torch

    from .. import MPI, Communicator

    comm = Communicator(MPI.COMM_WORLD)
    torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
    dev = comm.dev
    rank, p = comm.Get_rank(), comm.Get_size()
    want = p * (p + 1) / 2
    bad = []
    for dt in (torch.float32, torch.bfloat16):
        x = dev.empty(1 << 20, dt)
        y = dev.empty(1 << 20, dt)
        for algo in ("twoshot", "fanout"):
            x.fill_(rank + 1)
            dev.allreduce(x, y, "SUM", algo, symmetric=True)
            torch.cuda.synchronize()
            got = y.float()
            if not bool((got == want).all()):
                bad.append(f"{algo} {dt}: {got.min().item()}..{got.max().item()} != {want}")
    dev.check()
    bad = comm.comm.allgather(bad)
    if rank == 0:
        flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
        print("\n".join(flat) if flat else "multi-rank smoke OK", flush=True)
    return 1 if any(bad) else 0


if __name__ == "__main__":
    sys.exit(main())
