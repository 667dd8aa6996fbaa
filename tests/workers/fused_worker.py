"""Fused row-parallel GEMM + TP all-reduce (DeviceGroup.gemm_allreduce) on p ranks.

Every rank holds a K-shard x_r [M, K/p], w_r [N, K/p] (seeded per rank, so every rank
regenerates all shards); the output must equal sum_r x_r w_r^T (+ bias):
* against an fp32 reference of the whole product (bf16 tolerance);
* bitwise against the unfused path on the same four-wave kernel (gemm_nt, then the
  rank-order fan-out all-reduce of the bf16 partials), without bias;
* identical on every rank (one reducer writes every rank's tile);
* over repeated calls, changing shapes (edge tiles, tile counts) and random per-rank
  delays (arrival order of the tile tickets);
* RowParallelLinear forward/backward through the fused path vs the unfused layer.
Prints "fused OK" on success."""
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
dev = comm.dev
D = dev.device
fails = []


def shard(r, rows, cols, salt):
    g = torch.Generator(device=D).manual_seed(7919 * r + 104729 * salt + 1)
    return (torch.rand(rows, cols, generator=g, device=D) * 2 - 1).bfloat16()


rng = random.Random(31 + rank)
for salt, (M, N, Kr, use_bias) in enumerate([(512, 768, 256, False), (300, 520, 128, True), (1024, 1024, 512, False),
                                              (256, 256, 64, True), (777, 1032, 192, False), (2048, 4096, 1024, True)]):
    xs = [shard(r, M, Kr, salt) for r in range(p)]
    ws = [shard(r + 100, N, Kr, salt) for r in range(p)]
    bias = (torch.rand(N, device=D, generator=torch.Generator(device=D).manual_seed(salt)) - 0.5) if use_bias else None
    ref = sum(xs[r].float() @ ws[r].float().T for r in range(p))
    if bias is not None:
        ref = ref + bias
    for rep in range(3):
        if rng.random() < 0.5:
            time.sleep(rng.random() * 0.02)  # host skew: ranks reach the kernel in random order
        y = dev.gemm_allreduce(xs[rank], ws[rank], bias=bias)
        torch.cuda.synchronize()
        dev.check()
        err = (y.float() - ref).abs().max().item()
        tol = 0.02 * (Kr * p) ** 0.5 + 0.02
        if err > tol:
            fails.append(f"fused[{M}x{N}x{Kr},bias={use_bias},rep={rep}]: max err {err:.4f} > {tol:.4f}")
        # identical on every rank
        h = float(y.float().sum().item())
        hs = comm.comm.allgather(h)
        if any(x != hs[0] for x in hs):
            fails.append(f"fused[{M}x{N}x{Kr}]: outputs differ between ranks {hs}")
    if not use_bias:
        # bitwise vs gemm_nt on the same kernel + rank-order fan-out all-reduce of the bf16 partials
        D_ = _native.device()
        D_.gemm_set_kernel(5)
        part = gemm_nt(xs[rank], ws[rank])
        D_.gemm_set_kernel(0)
        unf = torch.empty_like(part)
        dev.allreduce(part, unf, "SUM", "fanout")
        torch.cuda.synchronize()
        if not torch.equal(unf, y):
            diff = (unf.float() - y.float()).abs().max().item()
            fails.append(f"fused[{M}x{N}x{Kr}] != unfused rank-order sum (max diff {diff})")

# RowParallelLinear through every row-parallel mode (same weights): the fused epilogue,
# the chunked side-stream overlap and the plain path must agree with an fp32 reference,
# and each mode must really take its own path (tp.CALLS counts the paths that ran)
from collective_communication_mpi_amd.parallel import tensor_parallel as tp  # noqa: E402

IN, OUT, T = 256 * p, 512, 1024  # every rank holds a K shard of 256 (the fused path needs K_r % 64 == 0)
x_full = shard(999, T, IN, 77)
layer = tp.RowParallelLinear(IN, OUT, comm, bias=True, input_is_parallel=False, device=D, dtype=torch.bfloat16, seed=5)
wf = tp.full_weight(layer, comm).to(D)
xr = x_full.float().requires_grad_(True)
yr = xr @ wf.T + layer.bias.float()
yr.pow(2).sum().backward()
grads = {}
for mode, path in (("fused", "row_fused"), ("chunked", "row_chunked"), ("plain", "row_plain")):
    layer.mode = mode
    layer.zero_grad()
    before = tp.CALLS[path]
    xin = x_full.clone().requires_grad_(True)
    y = layer(xin)
    y.float().pow(2).sum().backward()
    torch.cuda.synchronize()
    if tp.CALLS[path] != before + 1:
        fails.append(f"RowParallelLinear mode {mode}: path {path} ran {tp.CALLS[path] - before} times, expected 1")
    err = ((y.float() - yr).abs().max() / yr.abs().max()).item()
    if err > 0.02:
        fails.append(f"RowParallelLinear {mode} forward vs fp32: rel err {err:.4f}")
    grads[mode] = (xin.grad.clone(), layer.weight.grad.clone(), layer.bias.grad.clone())
for mode, (gx, gw, gb) in grads.items():
    for name, a_, b_ in (("dx", gx, xr.grad), ("dw", gw, None), ("db", gb, None)):
        if b_ is None:
            a_ref = grads["plain"][1] if name == "dw" else grads["plain"][2]
            rel = ((a_.float() - a_ref.float()).abs().max() / (a_ref.float().abs().max() + 1e-6)).item()
        else:
            rel = ((a_.float() - b_.float()).abs().max() / (b_.float().abs().max() + 1e-6)).item()
        if rel > 0.05:
            fails.append(f"RowParallelLinear {mode} {name}: rel err {rel:.4f}")

torch.cuda.synchronize()
dev.check()
bad = comm.comm.allreduce(len(fails), op=MPI.SUM)
if fails:
    print(f"[rank {rank}] " + "\n".join(fails[:20]), flush=True)
if rank == 0:
    print("fused OK" if bad == 0 else f"fused FAILED ({bad})", flush=True)
sys.exit(1 if bad else 0)
