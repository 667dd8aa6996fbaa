"""Routes of the Llama-3-8B MLP backward's weight-gradient GEMMs.

dW = dY^T X with both operands M-major (K = tokens):
* ``transpose``: both operands transposed (k_transpose16), then the N-layout pair ring
  (round 4's route: 3 transposes per MLP step);
* ``kmajor``: only dY transposed (or its N-layout copy taken from the producer: the SwiGLU
  backward writes dh^T), X read K-major by the pair ring's TB form (no transpose of X);
* ``pair``: both operands read K-major by the pair ring's TA + TB form: no transposes, and
  the SwiGLU backward writes no dh^T (CCMPI_KMAJOR_ROUTE=pair).

Times each dW GEMM both ways (CUDA events, median), checks them against fp32, then the
whole ParallelSwiGLUMLP forward + backward at TP = 1 with each route (CCMPI_WGRAD_B), and
prints one JSON line per measurement.

    python benchmarks/mlp_bwd_routes.py [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_ring  # noqa: E402
from collective_communication_mpi_amd.parallel.mlp_bench import measure_tp_mlp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--tokens", type=int, default=4096)
args = ap.parse_args()


def t_ms(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(args.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


T, d, f = args.tokens, 4096, 14336
g = torch.Generator(device="cuda").manual_seed(0)
for name, (n_out, k_in) in {"down": (d, f), "gate_up": (2 * f, d)}.items():
    x = (torch.rand(T, k_in, device="cuda", generator=g) * 2 - 1).bfloat16()
    dy = (torch.rand(T, n_out, device="cuda", generator=g) * 2 - 1).bfloat16()
    dyt = dy.t().contiguous()  # the producer-written N-layout copy (gate_up: dh^T from the SwiGLU backward)
    ref = dy.float().T @ x.float()
    rec = {"gemm": f"dW_{name}", "shape": [n_out, k_in, T]}
    for route in ("transpose", "kmajor", "pair"):
        os.environ["CCMPI_KMAJOR_ROUTE"] = "pair" if route == "pair" else "transpose"
        os.environ["CCMPI_WGRAD_B"] = route if route != "pair" else "kmajor"
        for src, a_nt in ((("dY_transposed_here", None), ("dYT_given", dyt)) if route != "pair"
                          else (("no_transposes", None),)):
            got = gemm_ring(dy, x, True, True, a_nt=a_nt)
            err = ((got.float() - ref).abs().max() / ref.abs().max()).item()
            ms = t_ms(lambda: gemm_ring(dy, x, True, True, a_nt=a_nt))
            rec[f"{route}/{src}_ms"] = round(ms, 4)
            rec[f"{route}/{src}_TFLOPs"] = round(2 * T * n_out * k_in / ms / 1e9, 1)
            rec[f"{route}/{src}_rel_err"] = round(err, 5)
    print(json.dumps(rec), flush=True)

comm = Communicator(MPI.COMM_WORLD)
for route in ("transpose", "kmajor", "pair"):
    os.environ["CCMPI_KMAJOR_ROUTE"] = "pair" if route == "pair" else "transpose"
    os.environ["CCMPI_WGRAD_B"] = route if route != "pair" else "kmajor"
    r = measure_tp_mlp(comm, tokens=T, iters=10, warmup=3)
    print(json.dumps({"mlp_route": route, **{k: r[k] for k in ("fwd_ms", "fwd_bwd_ms", "fwd_bwd_TFLOPs", "tp_paths",
                                                               "out_abs_mean")}}), flush=True)
