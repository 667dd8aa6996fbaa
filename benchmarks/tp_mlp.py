"""Tensor-parallel Llama-3-8B MLP block on the generic TP layers (parallel/tensor_parallel.py).

    python benchmarks/tp_mlp.py                          # TP = 1 (whole block on one rank)
    scripts/mpirun -n 2 python benchmarks/tp_mlp.py      # TP = 2 (ranks sharing the GPU, or one per GPU)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/tp_mlp.py

The block is ``y = W_down (silu(W_gate x) * W_up x)`` with d = 4096, ffn = 14336, bf16, as
``ParallelSwiGLUMLP``: a ``ColumnParallelLinear`` gate|up (interleaved (gate, up) rows,
2 x 14336 / p output features per rank, the SwiGLU gate in the GEMM's epilogue, Megatron
"f": dX all-reduced in backward) and a ``RowParallelLinear`` down (Megatron "g": one TP
all-reduce of the T x 4096 output in forward).  Times forward and forward + backward over
``--tokens`` tokens (median of ``--iters``, max over ranks), the TP all-reduce of the same
T x 4096 bf16 tensor alone, and reports the model TFLOP/s of the whole group
(``parallel/mlp_bench.py``).  One JSON line from rank 0.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel.mlp_bench import measure_tp_mlp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=int, default=4096)
ap.add_argument("--d", type=int, default=4096)
ap.add_argument("--ffn", type=int, default=14336)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--eager-gate", action="store_true",
                help="SwiGLU gate as eager torch ops (A/B against the gate fused into the GEMM epilogue)")
ap.add_argument("--variants", action="store_true", help="p > 1: every row-parallel mode side by side")
ap.add_argument("--mode", default="", help="row-parallel mode of the main record (plain | chunked | fused | push)")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
res = measure_tp_mlp(comm, tokens=args.tokens, d=args.d, ffn=args.ffn, iters=args.iters, warmup=args.warmup,
                     eager_gate=args.eager_gate, variants=args.variants, mode=args.mode)
if comm.Get_rank() == 0:
    print(json.dumps({"bench": "tp_mlp", **res}), flush=True)
