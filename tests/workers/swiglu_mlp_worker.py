"""ParallelSwiGLUMLP over a TP group of every rank vs a single-process fp32 reference.

    scripts/mpirun -n 2 python tests/workers/swiglu_mlp_worker.py --device cpu
    scripts/mpirun -n 2 python tests/workers/swiglu_mlp_worker.py --device cuda

Forward output on every rank, dX, and the gate|up / down weight gradients (reassembled
from the shards: rank r holds gate and up rows [r k, (r+1) k) as interleaved pairs) against
fp32 autograd of ``W_down (silu(W_gate x) * W_up x)`` with the unsharded weights.
Prints "swiglu mlp OK" on success."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel.tensor_parallel import ParallelSwiGLUMLP, _init_full  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--device", default="cpu")
args = ap.parse_args()

comm = Communicator(MPI.COMM_WORLD)
hc = comm.comm
rank, p = comm.Get_rank(), comm.Get_size()
if args.device == "cuda":
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
    torch.cuda.set_device(local % torch.cuda.device_count())
    dev, dt, tol = torch.device("cuda", torch.cuda.current_device()), torch.bfloat16, 0.05
else:
    dev, dt, tol = torch.device("cpu"), torch.float32, 1e-4

D, F, T = 128, 64 * p, 48
mlp = ParallelSwiGLUMLP(D, F, comm, device=dev, dtype=dt, seed=11)
gen = torch.Generator().manual_seed(3)
x0 = torch.randn(T, D, generator=gen)
gy = torch.randn(T, D, generator=gen) * 0.1

x = x0.to(dt).to(dev).requires_grad_(True)
y = mlp(x)
y.backward(gy.to(dt).to(dev))

# fp32 reference with the unsharded weights (the layers draw them from the same seeds)
wgu, _ = _init_full(2 * F, D, 11, torch.float32, False)
wd, _ = _init_full(D, F, 12, torch.float32, False)
wgu = wgu.to(dt).float().requires_grad_(True)
wd = wd.to(dt).float().requires_grad_(True)
xr = x0.to(dt).float().requires_grad_(True)
h = xr @ wgu.T
yr = (torch.nn.functional.silu(h[:, :F]) * h[:, F:]) @ wd.T
yr.backward(gy.to(dt).float())

fails = []


def rel(a, b):
    return ((a.float().cpu() - b).abs().max() / (b.abs().max() + 1e-6)).item()


if rel(y.detach(), yr.detach()) > tol:
    fails.append(f"forward rel err {rel(y.detach(), yr.detach())}")
if rel(x.grad, xr.grad) > tol:
    fails.append(f"dx rel err {rel(x.grad, xr.grad)}")
k = F // p
gu = hc.allgather(mlp.gate_up.weight.grad.detach().float().cpu())
g_full = torch.cat([s[0::2] for s in gu] + [s[1::2] for s in gu])  # shards interleave (gate j, up j) rows
if rel(g_full, wgu.grad) > tol:
    fails.append(f"d W_gate_up rel err {rel(g_full, wgu.grad)}")
gd = torch.cat(hc.allgather(mlp.down.weight.grad.detach().float().cpu()), dim=1)
if rel(gd, wd.grad) > tol:
    fails.append(f"d W_down rel err {rel(gd, wd.grad)}")

bad = hc.allgather(fails)
if rank == 0:
    flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
    print("\n".join(flat) if flat else "swiglu mlp OK", flush=True)
sys.exit(1 if any(bad) else 0)
