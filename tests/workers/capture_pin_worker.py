"""a registration slot a captured HIP graph resolves must survive later
registrations.  CCMPI_REGISTER_SLOTS=2; an all-reduce on ordinary (registered-on-demand)
tensors is captured, then more distinct allocations than there are slots are all-reduced
eagerly (LRU pressure), then the graph is replayed on new input values and must produce
their exact sum.  Prints "capture pin OK"."""
import os
import sys

os.environ["CCMPI_REGISTER_SLOTS"] = "2"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
rank, p = comm.Get_rank(), comm.Get_size()
dev = comm.dev
fails = []
n = (12 << 20) // 4  # > 10 MiB: its own caching-allocator segment
x = torch.empty(n, device=dev.device)
y = torch.empty(n, device=dev.device)
x.fill_(rank + 1.0)
dev.allreduce(x, y, "SUM", "fanout")  # eager: maps the slot(s) of x and y
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        dev.allreduce(x, y, "SUM", "fanout")  # slot hit during capture: pinned
torch.cuda.synchronize()
if not dev._pinned:
    fails.append("capture pinned no slot")
regs0 = dev.registrations
others = [torch.full((n,), float(rank + 1), device=dev.device) for _ in range(4)]
outs = [torch.empty(n, device=dev.device) for _ in range(4)]
for a, b in zip(others, outs):
    dev.allreduce(a, b, "SUM", "fanout")  # new allocations: LRU pressure on 2 slots
torch.cuda.synchronize()
if dev.registrations <= regs0:
    fails.append("no new registrations under LRU pressure")
for b in outs:
    if not torch.all(b == p * (p + 1) / 2).item():
        fails.append("eager all-reduce under LRU pressure wrong")
        break
x.fill_(rank + 2.0)
y.zero_()
torch.cuda.synchronize()
comm.comm.Barrier()
g.replay()
torch.cuda.synchronize()
dev.check()
want = p * (p + 1) / 2 + p
if not torch.all(y == want).item():
    fails.append(f"graph replay after LRU pressure: got {y[:4].tolist()} want {want}")
bad = comm.comm.allgather(fails)
if rank == 0:
    flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
    print("\n".join(flat) if flat else "capture pin OK", flush=True)
sys.exit(1 if any(bad) else 0)
