"""Multi-rank check of the generic tensor-parallel layers + bucketed DDP against a
single-process fp32 reference (every rank computes the reference itself from
the same seeds, so no extra communication is needed to check).

    scripts/mpirun -n 4 python tests/workers/tp_ddp_worker.py --device cpu
    scripts/mpirun -n 2 python tests/workers/tp_ddp_worker.py --device cuda

Model (mp-major grid from get_info, TP = 2 when the world is even):
  ColumnParallelLinear(D->H) -> GELU -> RowParallelLinear(H->D)
  -> ColumnParallelLinear(D->H, gather_output) -> RowParallelLinear(H->D, input_is_parallel=False)
DDP over the DP communicator with tiny buckets (several buckets, overlap path);
two SGD steps, the second after zero_grad(set_to_none=True).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator, get_info  # noqa: E402
from collective_communication_mpi_amd.parallel import (  # noqa: E402
    ColumnParallelLinear, DistributedDataParallel, RowParallelLinear)
from collective_communication_mpi_amd.parallel.tensor_parallel import _init_full, full_weight  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--device", default="cpu")
ap.add_argument("--schedule", default=None, help="DDP schedule: overlap | deferred | auto (default)")
ap.add_argument("--steps", type=int, default=2, help="SGD steps (auto needs 6 to decide)")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
rank, world = comm.Get_rank(), comm.Get_size()
tp = 2 if world % 2 == 0 else 1
dp = world // tp
D, H, S, per = 64, 128, 4, 3
mp_idx, dp_idx, mp_comm, dp_comm, _, _ = get_info(comm, rank, tp, dp, "fc_q", D, H)
cuda = args.device == "cuda"
if cuda:
    torch.cuda.set_device(0 if torch.cuda.device_count() == 1 else rank % torch.cuda.device_count())
dev = torch.device("cuda" if cuda else "cpu")
dt = torch.bfloat16 if cuda else torch.float32
tol = 6e-2 if cuda else 2e-5


class TPModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        kw = dict(device=dev, dtype=dt)
        self.c1 = ColumnParallelLinear(D, H, mp_comm, seed=1, **kw)
        self.r1 = RowParallelLinear(H, D, mp_comm, seed=2, **kw)
        self.c2 = ColumnParallelLinear(D, H, mp_comm, gather_output=True, seed=3, **kw)
        self.r2 = RowParallelLinear(H, D, mp_comm, input_is_parallel=False, seed=4, **kw)

    def forward(self, x):
        return self.r2(self.c2(self.r1(torch.nn.functional.gelu(self.c1(x)))))


class RefModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.ls = torch.nn.ModuleList()
        for seed, (i, o) in zip((1, 2, 3, 4), ((D, H), (H, D), (D, H), (H, D))):
            lin = torch.nn.Linear(i, o)
            w, b = _init_full(o, i, seed, torch.float32, True)
            with torch.no_grad():
                lin.weight.copy_(w.to(dt).float())
                lin.bias.copy_(b.to(dt).float())
            self.ls.append(lin)

    def forward(self, x):
        c1, r1, c2, r2 = self.ls
        return r2(c2(r1(torch.nn.functional.gelu(c1(x)))))


def rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / b.float().cpu().norm().clamp_min(1e-12)).item()


model = DistributedDataParallel(TPModel(), dp_comm, bucket_bytes=16 << 10, schedule=args.schedule)
ref = RefModel()
opt = torch.optim.SGD(model.parameters(), lr=0.05)
ropt = torch.optim.SGD(ref.parameters(), lr=0.05)
g = torch.Generator().manual_seed(123)
fails = []
for step in range(args.steps):
    xg = torch.randn(dp * per, S, D, generator=g)                 # global batch
    xl = xg[dp_idx * per:(dp_idx + 1) * per]                      # this DP replica's block (split_data)
    if step == 0:
        model.zero_grad()
    else:
        opt.zero_grad(set_to_none=True)
    out = model(xl.to(dev, dt))
    loss = (out.float() ** 2).mean()
    loss.backward()
    model.finish()
    ropt.zero_grad()
    rout = ref(xg.to(dt).float())
    (rout ** 2).mean().backward()
    e_out = rel(out, rout[dp_idx * per:(dp_idx + 1) * per])
    if e_out > tol:
        fails.append(f"step {step} forward rel err {e_out:.2e}")
    for name, lyr, rl in (("c1", model.module.c1, ref.ls[0]), ("r1", model.module.r1, ref.ls[1]),
                          ("c2", model.module.c2, ref.ls[2]), ("r2", model.module.r2, ref.ls[3])):
        dim = 0 if isinstance(lyr, ColumnParallelLinear) else 1
        gparts = mp_comm.comm.allgather(lyr.weight.grad.detach().float().cpu()) if tp > 1 else [
            lyr.weight.grad.detach().float().cpu()]
        gfull = torch.cat(gparts, dim=dim)
        e = rel(gfull, rl.weight.grad)
        if e > tol:
            fails.append(f"step {step} {name} weight grad rel err {e:.2e}")
    opt.step()
    ropt.step()
for name, lyr, rl in (("c1", model.module.c1, ref.ls[0]), ("r2", model.module.r2, ref.ls[3])):
    e = rel(full_weight(lyr, mp_comm), rl.weight.detach())
    if e > tol:
        fails.append(f"{name} weight after 2 SGD steps rel err {e:.2e}")
if args.schedule == "auto" and args.steps >= 6 and world // tp > 1 and cuda:
    if not model.schedule_choice or model.schedule_choice["chosen"] != model.schedule:
        fails.append(f"auto schedule undecided after {args.steps} steps: {model.schedule_choice}")
if len(model.buckets) < 2:
    fails.append(f"expected several buckets, got {model.bucket_sizes}")
comm.Barrier()
if fails:
    print(f"[rank {rank}] FAIL: {fails}", flush=True)
    sys.exit(1)
if rank == 0:
    print(f"tp/ddp OK world={world} tp={tp} dp={dp} device={args.device} buckets={len(model.buckets)} "
          f"schedule={model.schedule} choice={model.schedule_choice}", flush=True)
