"""Backward GEMMs of the Llama-3-8B TP MLP on the LDS-ring kernel with K-major operands
(dX = dY W: NN, dW = dY^T X: TN) against hipBLASLt and the older routes (explicit
transpose + NT kernel, 256x256 TN kernel).  Median of --iters CUDA-event timings.

    python benchmarks/gemm_ring_bench.py [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_nt, gemm_ring, gemm_tn, transpose  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
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


T, d, f = 4096, 4096, 14336
rows = []
g = torch.Generator(device="cuda").manual_seed(0)
for name, (tok, nout, kin) in {"gate_up": (T, 2 * f, d), "down": (T, d, f)}.items():
    x = (torch.rand(tok, kin, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(nout, kin, device="cuda", generator=g) * 2 - 1) / kin ** 0.5).bfloat16()
    dy = (torch.rand(tok, nout, device="cuda", generator=g) * 2 - 1).bfloat16()
    macs = tok * nout * kin
    # dX = dY W  [tok, kin]
    ref = dy.float() @ w.float()
    got = gemm_ring(dy, w, False, True)
    err = (got.float() - ref).abs().max().item()
    r = {"layer": name, "gemm": "dX", "shape": [tok, kin, nout], "ring_max_err": err,
         "ring_ms": t_ms(lambda: gemm_ring(dy, w, False, True)),
         "transpose_nt_ms": t_ms(lambda: gemm_nt(dy, transpose(w))),
         "hipblaslt_ms": t_ms(lambda: dy @ w)}
    rows.append(r)
    # dW = dY^T X  [nout, kin]
    ref = dy.float().T @ x.float()
    got = gemm_ring(dy, x, True, True)
    err = (got.float() - ref).abs().max().item()
    r = {"layer": name, "gemm": "dW", "shape": [nout, kin, tok], "ring_max_err": err,
         "ring_ms": t_ms(lambda: gemm_ring(dy, x, True, True)),
         "tn256_fp32_ms": t_ms(lambda: gemm_tn(dy, x)),
         "hipblaslt_ms": t_ms(lambda: dy.T @ x)}
    rows.append(r)
    for r in rows[-2:]:
        for k in [k for k in r if k.endswith("_ms")]:
            r[k.replace("_ms", "_tflops")] = round(2 * macs / (r[k] * 1e-3) / 1e12, 1)
for r in rows:
    print(json.dumps(r))
