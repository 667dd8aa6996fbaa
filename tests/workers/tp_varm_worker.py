"""the TP layers' persistent scratch (row-parallel partial, dX partial) is one
grow-only symmetric-heap block per role -- token counts that vary across steps (eval,
packing, a last partial batch) reuse it instead of allocating a block per shape.  A
ParallelSwiGLUMLP over every rank runs forward + backward at varying M: every output matches
fp32 autograd, and once the largest M has been seen the device plane makes no more host
calls (no new heap blocks).  Prints "varm OK"."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel import tensor_parallel as tp  # noqa: E402
from collective_communication_mpi_amd.parallel.tensor_parallel import ParallelSwiGLUMLP, _init_full  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
hc = comm.comm
p = comm.Get_size()
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
dev = torch.device("cuda", torch.cuda.current_device())
D, F = 256, 128 * p
mlp = ParallelSwiGLUMLP(D, F, comm, device=dev, dtype=torch.bfloat16, seed=11)
wgu, _ = _init_full(2 * F, D, 11, torch.float32, False)
wd, _ = _init_full(D, F, 12, torch.float32, False)
wgu, wd = wgu.bfloat16().float(), wd.bfloat16().float()
fails = []
dg = tp.device_group_for(comm)
calls_after_max = None
for step, T in enumerate([512, 256, 1024, 128, 768, 1024, 256, 512]):
    g = torch.Generator().manual_seed(step)
    x0 = torch.randn(T, D, generator=g).bfloat16()
    x = x0.to(dev).requires_grad_(True)
    y = mlp(x)
    y.backward(torch.ones_like(y) * 0.01)
    torch.cuda.synchronize()
    xr = x0.float().requires_grad_(True)
    h = xr @ wgu.T
    yr = (torch.nn.functional.silu(h[:, :F]) * h[:, F:]) @ wd.T
    yr.backward(torch.ones_like(yr).bfloat16().float() * 0.01)
    err = ((y.float().cpu() - yr.detach()).abs().max() / yr.abs().max()).item()
    errx = ((x.grad.float().cpu() - xr.grad).abs().max() / xr.grad.abs().max()).item()
    if err > 0.05 or errx > 0.05:
        fails.append(f"T={T}: rel err y {err:.4f} dx {errx:.4f}")
    if T == 1024 and calls_after_max is None:
        calls_after_max = dg.host_calls
mlp.gate_up.weight.grad = None
if dg.host_calls != calls_after_max:
    fails.append(f"host calls grew after the largest M: {calls_after_max} -> {dg.host_calls}")
grow = [k for k in dg._persist if k[0] == "grow"]
if len({k[1] for k in grow}) != len(grow):
    fails.append(f"more than one scratch block per role: {grow}")
bad = hc.allgather(fails)
if comm.Get_rank() == 0:
    flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
    print("\n".join(flat) if flat else "varm OK", flush=True)
sys.exit(1 if any(bad) else 0)
