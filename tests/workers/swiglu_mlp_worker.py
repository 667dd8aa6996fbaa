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
ap.add_argument("--big", action="store_true",
                help="shapes that take the LDS-ring GEMM and its SwiGLU epilogue (with CCMPI_SHARED_RING=1 "
                     "and CCMPI_RING_MIN_MACS=1: beside the other ranks' collectives on one GPU)")
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

D, F, T = (1024, 512 * p, max(1024, 256 * p)) if args.big else (128, 64 * p, 48)  # push: T % (256 p)
if args.big and args.device == "cuda":
    from collective_communication_mpi_amd import _native  # noqa: E402

    ring0 = _native.device().gemm_ring_launches()
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

if args.big and args.device == "cuda" and _native.device().gemm_ring_launches() == ring0:
    fails.append("--big: no LDS-ring GEMM launched (the path under test did not run)")
if (args.big and args.device == "cuda" and os.environ.get("CCMPI_KMAJOR_MIN_MACS") == "1"
        and os.environ.get("CCMPI_KMAJOR_ROUTE") == "transpose"):
    from collective_communication_mpi_amd.parallel import tensor_parallel as _tp  # noqa: E402

    if not _tp.CALLS["dh_transposed"]:
        fails.append("--big: the dW transpose route (dh^T from the SwiGLU backward) did not run")

if args.big and args.device == "cuda" and p > 1 and os.environ.get("CCMPI_SHARED_RING") == "1":
    # the push row-parallel form (the GEMM epilogue stores each row block into its owner's
    # inbox, then an inbox-to-local two-shot): same bf16 partials and the same rank-order
    # reduction as plain, so the block's output must match plain bit for bit
    from collective_communication_mpi_amd.parallel import tensor_parallel as tp  # noqa: E402

    outs = {}
    dg = tp.device_group_for(comm)
    for mode in ("plain", "push"):
        m = ParallelSwiGLUMLP(D, F, comm, device=dev, dtype=dt, seed=11, mode=mode)
        for it in range(2):
            xi = x0.to(dt).to(dev).requires_grad_(True)
            c0, h0 = tp.CALLS["row_" + mode], dg.host_calls
            yi = m(xi)
            yi.backward(gy.to(dt).to(dev))
            torch.cuda.synchronize()
            if tp.CALLS["row_" + mode] != c0 + 1:
                fails.append(f"{mode}: row path did not run ({dict(tp.CALLS)})")
            if it == 1 and dg.host_calls != h0:
                fails.append(f"{mode}: steady-state step made {dg.host_calls - h0} host calls (expected 0)")
        outs[mode] = (yi.detach().clone(), xi.grad.clone())
    if not torch.equal(outs["push"][0], outs["plain"][0]):
        fails.append(f"push: forward differs from plain (max {(outs['push'][0].float() - outs['plain'][0].float()).abs().max().item()})")
    if rel(outs["push"][1], xr.grad) > tol:
        fails.append(f"push: dx rel err {rel(outs['push'][1], xr.grad)}")
    # the DeviceGroup call itself against an fp32 sum of every rank's product, 2 shapes
    for (M2, N2, K2) in ((256 * p, 512, 128), (512 * p, 1032, 192)):
        ga = torch.Generator().manual_seed(40 + rank)
        xa = (torch.randn(M2, K2, generator=ga) * 0.5).to(dt)
        wa = (torch.randn(N2, K2, generator=ga) * 0.5).to(dt)
        ref = sum(a.float() @ b.float().T for a, b in hc.allgather((xa, wa)))
        out = torch.empty(M2, N2, dtype=dt, device=dev)
        dg.gemm_push_allreduce(xa.to(dev), wa.to(dev), out)
        if rel(out, ref) > 0.02:
            fails.append(f"gemm_push_allreduce {M2}x{N2}x{K2}: rel err {rel(out, ref)}")
    try:
        dg.gemm_push_allreduce(xa[:300].to(dev), wa.to(dev), torch.empty(300, N2, dtype=dt, device=dev))
        fails.append("gemm_push_allreduce accepted M % (256 p) != 0")
    except (ValueError, RuntimeError):
        pass

if args.device == "cuda" and p > 1 and not args.big:
    # every row-parallel mode through the whole block (forward + backward), its path
    # really taken, and a steady-state step with no host call from the device plane
    from collective_communication_mpi_amd.parallel import tensor_parallel as tp  # noqa: E402

    T2 = 512  # two 256-row blocks for the chunked mode
    x2 = torch.randn(T2, D, generator=torch.Generator().manual_seed(5))
    g2 = torch.randn(T2, D, generator=torch.Generator().manual_seed(6)) * 0.1
    xr2 = x2.to(dt).float().requires_grad_(True)
    h2 = xr2 @ wgu.detach().T
    yr2 = (torch.nn.functional.silu(h2[:, :F]) * h2[:, F:]) @ wd.detach().T
    yr2.backward(g2.to(dt).float())
    for mode, path in (("plain", "row_plain"), ("chunked", "row_chunked"), ("fused", "row_fused")):
        m = ParallelSwiGLUMLP(D, F, comm, device=dev, dtype=dt, seed=11, mode=mode)
        dg = tp.device_group_for(comm)
        for it in range(2):
            xi = x2.to(dt).to(dev).requires_grad_(True)
            c0, b0, h0 = tp.CALLS[path], tp.CALLS["col_bwd_overlap"], dg.host_calls
            yi = m(xi)
            yi.backward(g2.to(dt).to(dev))
            torch.cuda.synchronize()
            if tp.CALLS[path] != c0 + 1 or tp.CALLS["col_bwd_overlap"] != b0 + 1:
                fails.append(f"{mode}: paths {dict(tp.CALLS)} (expected one {path} and one col_bwd_overlap)")
            if it == 1 and dg.host_calls != h0:
                fails.append(f"{mode}: steady-state step made {dg.host_calls - h0} host calls (expected 0)")
        if rel(yi.detach(), yr2.detach()) > tol:
            fails.append(f"{mode}: forward rel err {rel(yi.detach(), yr2.detach())}")
        if rel(xi.grad, xr2.grad) > tol:
            fails.append(f"{mode}: dx rel err {rel(xi.grad, xr2.grad)}")

bad = hc.allgather(fails)
if rank == 0:
    flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
    print("\n".join(flat) if flat else "swiglu mlp OK", flush=True)
sys.exit(1 if any(bad) else 0)
