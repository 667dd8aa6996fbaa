"""Tensor-parallel Llama-3-8B MLP block on the generic TP layers (parallel/tensor_parallel.py).

    python benchmarks/tp_mlp.py                          # TP = 1 (whole block on one rank)
    scripts/mpirun -n 2 python benchmarks/tp_mlp.py      # TP = 2 (ranks sharing the GPU, or one per GPU)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/tp_mlp.py

The block is ``y = W_down (silu(W_gate x) * W_up x)`` with d = 4096, ffn = 14336, bf16:
``ColumnParallelLinear`` (gate | up, 2 x 14336 / p output features per rank, Megatron "f":
dX all-reduced in backward) -> SiLU-gate -> ``RowParallelLinear`` (14336 / p input features,
Megatron "g": one TP all-reduce of the T x 4096 output in forward).  GEMMs on the MFMA bf16
kernels.  Times forward and forward + backward over ``--tokens`` tokens (median of
``--iters``, max over ranks), the TP all-reduce of the same T x 4096 bf16 tensor alone, and
reports the model TFLOP/s of the whole group (the reference's TP forward,
model/func_impl.py:76-109, on a realistic layer shape).  One JSON line from rank 0.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel.tensor_parallel import (  # noqa: E402
    ParallelSwiGLUMLP, all_reduce_)

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=int, default=4096)
ap.add_argument("--d", type=int, default=4096)
ap.add_argument("--ffn", type=int, default=14336)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--eager-gate", action="store_true",
                help="SwiGLU gate as eager torch ops (A/B against the gate fused into the GEMM epilogue)")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
dev = torch.device("cuda", torch.cuda.current_device())
hc = comm.comm
T, d, f = args.tokens, args.d, args.ffn

mlp = ParallelSwiGLUMLP(d, f, comm, device=dev, dtype=torch.bfloat16, seed=1)
gate_up, down = mlp.gate_up, mlp.down
k = f // p


def block(x):
    if not args.eager_gate:
        return mlp(x)
    h = gate_up(x)
    a = torch.nn.functional.silu(h[:, 0::2]) * h[:, 1::2]  # shard rows are (gate, up) pairs
    return down(a)


x = (torch.randn(T, d, generator=torch.Generator().manual_seed(3)) * 0.5).to(torch.bfloat16).to(dev).requires_grad_(True)
gy = (torch.randn(T, d, generator=torch.Generator().manual_seed(4)) * 0.01).to(torch.bfloat16).to(dev)


def timed(fn):
    for _ in range(args.warmup):
        fn()
    ts = []
    for _ in range(args.iters):
        torch.cuda.synchronize()
        hc.Barrier()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return hc.allreduce(statistics.median(ts), op=MPI.MAX)


def fwd():
    with torch.no_grad():
        block(x)


def fwd_bwd():
    x.grad = None
    for prm in (gate_up.weight, down.weight):
        prm.grad = None
    block(x).backward(gy)


t_f = timed(fwd)
t_fb = timed(fwd_bwd)
buf = torch.randn(T, d, device=dev).to(torch.bfloat16)
t_ar = timed(lambda: all_reduce_(buf, comm)) if p > 1 else 0.0
# checksum of the forward output: identical across TP degrees up to bf16 rounding
with torch.no_grad():
    y = block(x)
chk = float(y.float().abs().mean().item())
flop_f = 2 * T * d * 2 * f + 2 * T * f * d  # whole block (all ranks together)
if rank == 0:
    print(json.dumps({
        "bench": "tp_mlp", "tp": p, "gate": "eager" if args.eager_gate else "fused", "tokens": T, "d_model": d, "ffn": f, "dtype": "bf16",
        "shared_gpu": comm.dev.shared_device if p > 1 else False,
        "fwd_ms": round(t_f * 1e3, 3), "fwd_bwd_ms": round(t_fb * 1e3, 3),
        "fwd_TFLOPs": round(flop_f / t_f / 1e12, 1), "fwd_bwd_TFLOPs": round(3 * flop_f / t_fb / 1e12, 1),
        "tp_allreduce_bytes": T * d * 2, "tp_allreduce_ms": round(t_ar * 1e3, 3),
        "out_abs_mean": round(chk, 6)}), flush=True)
