"""DP gradient all-reduce overlapped with backward (BASELINE config: "DP8
gradient all-reduce, Llama-3-8B-sized grad (~16 GB bf16) overlapped with
backward on 8xMI355X").

A synthetic backward over ``--layers`` Llama-3-8B decoder layers (d 4096, GQA
kv 1024, MLP 14336): per layer the seven weight-gradient GEMMs
dW = dY^T X (hand-written ``gemm_tn``, fp32 accumulate) write that layer's
gradients into a flat bf16 gradient buffer on the DP group's symmetric heap;
as soon as a layer's GEMMs are issued its bucket is all-reduced on a side
stream (``GradBuckets``), so communication overlaps the next layers' GEMMs.
Reports compute-only, comm-only and overlapped step times and the fraction of
communication hidden.  32 layers = 6.98 B weights = 14 GB of bf16 grads
(+ embeddings ~ 16 GB at full size).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/dp_grad_overlap.py --layers 32
    scripts/mpirun -n 2 python benchmarks/dp_grad_overlap.py --layers 2 --tokens 2048
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_tn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--tokens", type=int, default=4096, help="tokens per rank per step")
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--algo", default="auto")
ap.add_argument("--comm-priority", type=int, default=-1, help="side-stream priority (-1 = high, 0 = normal)")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
dev = comm.dev
hc = comm.comm
d, kv, ff, T = 4096, 1024, 14336, args.tokens
# (out_features, in_features) of each weight of one layer
shapes = [(d, d), (kv, d), (kv, d), (d, d), (ff, d), (ff, d), (d, ff)]
per_layer = sum(a * b for a, b in shapes)
grads = dev.empty(per_layer * args.layers, torch.float32)  # fp32 master grads
act_in = {k: torch.randn(T, k, device=dev.device).bfloat16() for k in {d, ff}}
act_out = {k: torch.randn(T, k, device=dev.device).bfloat16() for k in {d, kv, ff}}
side = torch.cuda.Stream(priority=args.comm_priority)
events = [torch.cuda.Event() for _ in range(args.layers)]


def backward(comm_on: bool, compute_on: bool = True):
    off = 0
    for layer in reversed(range(args.layers)):
        base = layer * per_layer
        if compute_on:
            o = base
            for (fo, fi) in shapes:
                gemm_tn(act_out[fo], act_in[fi], out=grads[o:o + fo * fi].view(fo, fi), accumulate=False)
                o += fo * fi
        if comm_on:
            events[layer].record()
            side.wait_event(events[layer])
            with torch.cuda.stream(side):
                seg = grads[base:base + per_layer]
                dev.allreduce(seg, seg, "SUM", args.algo)
        off += per_layer
    torch.cuda.current_stream().wait_stream(side)


def timed(**kw):
    backward(**kw)
    torch.cuda.synchronize()
    hc.Barrier()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        backward(**kw)
    torch.cuda.synchronize()
    return hc.allreduce((time.perf_counter() - t0) / args.iters, op=MPI.MAX)


t_compute = timed(comm_on=False)
t_comm = timed(comm_on=True, compute_on=False) if p > 1 else 0.0
t_both = timed(comm_on=True) if p > 1 else t_compute
dev.check()
if rank == 0:
    hidden = 0.0 if p == 1 or t_comm == 0 else max(0.0, min(1.0, (t_compute + t_comm - t_both) / t_comm))
    flops = 2 * T * per_layer * args.layers
    print(json.dumps({"bench": "dp_grad_overlap", "ranks": p, "layers": args.layers, "grad_bytes_fp32": per_layer * args.layers * 4,
                      "tokens_per_rank": T, "compute_ms": round(t_compute * 1e3, 3), "comm_ms": round(t_comm * 1e3, 3),
                      "overlapped_ms": round(t_both * 1e3, 3), "comm_hidden_fraction": round(hidden, 3),
                      "wgrad_TFLOPs": round(flops / t_compute / 1e12, 1), "shared_gpu": dev.shared_device}), flush=True)
