"""LL all-reduce phase timing (s_memrealtime stamps of CTA 0 / thread 0), diagnostics.

    scripts/mpirun -n 2 python benchmarks/ll_stamps.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
dev = comm.dev
rank, p = comm.Get_rank(), comm.Get_size()
x = dev.empty(1024, torch.float32)
y = dev.empty(1024, torch.float32)
x.fill_(rank + 1)
dbg = torch.zeros(32, dtype=torch.int64, device=dev.device)
dev.allreduce(x, y, "SUM", "ll")
torch.cuda.synchronize()
dev.dc.set_debug_stamps(dbg.data_ptr())
for it in range(5):
    comm.comm.Barrier()
    dev.allreduce(x, y, "SUM", "ll")
    torch.cuda.synchronize()
    t = dbg.cpu().tolist()
    rel = [round((v - t[0]) / 100.0, 2) for v in t[:2 + p] + [t[16]]]  # 100 MHz ticks -> us
    print(f"rank {rank} it {it}: start 0, pushed {rel[1]}, sources {rel[2:2 + p]}, end {rel[-1]} us; ok={bool(torch.all(y == p * (p + 1) / 2))}", flush=True)
dev.dc.set_debug_stamps(0)
