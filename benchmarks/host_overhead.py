"""Host-side cost of one device all-reduce call, p ranks.

    python -m collective_communication_mpi_amd.launch -n 8 python benchmarks/host_overhead.py

For a 32 MiB bf16 tensor (the Llama TP all-reduce size at 4096 tokens):
* ``registered``: an ordinary torch tensor -- on-demand registration, one pickled host
  all-gather per call (the round-3 path of every TP all-reduce);
* ``heap``: symmetric-heap blocks, symmetric decided collectively (one host all-gather);
* ``heap_promise``: the same with ``symmetric=True`` (DDP buckets, the bench) -- no host call;
* ``to_local``: heap scratch reduced into an ordinary tensor (``allreduce_to_local``, the
  TP layers' path now) -- no host call.
Per variant: host microseconds per call (issue only: the loop queues ``--calls`` calls,
then one sync), the device plane's host calls per call, and wall time per call.  Rank 0
prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

calls = int(os.environ.get("CALLS", "50"))
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
dev, hc = comm.dev, comm.comm
n = (32 << 20) // 2
plain = torch.ones(n, dtype=torch.bfloat16, device=dev.device)
heap = dev.empty(n, torch.bfloat16)
heap2 = dev.empty(n, torch.bfloat16)
out = torch.empty(n, dtype=torch.bfloat16, device=dev.device)
variants = {
    "registered": lambda: dev.allreduce(plain, plain, "SUM", "fanout"),
    "heap": lambda: dev.allreduce(heap, heap2, "SUM", "fanout"),
    "heap_promise": lambda: dev.allreduce(heap, heap2, "SUM", "fanout", symmetric=True),
    "to_local": lambda: dev.allreduce_to_local(heap, out),
}
res = {}
for name, fn in variants.items():
    heap.fill_(1)
    fn()
    torch.cuda.synchronize()
    hc.Barrier()
    h0 = dev.host_calls
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    hcalls = (dev.host_calls - h0) / calls
    res[name] = {"host_us_per_call": round(hc.allreduce(t_issue, op=MPI.MAX) / calls * 1e6, 1),
                 "wall_us_per_call": round(hc.allreduce(t_all, op=MPI.MAX) / calls * 1e6, 1),
                 "host_calls_per_call": hcalls}
if comm.Get_rank() == 0:
    print(json.dumps({"ranks": comm.Get_size(), "bytes": n * 2, "shared_gpu": dev.shared_device, **res}), flush=True)
