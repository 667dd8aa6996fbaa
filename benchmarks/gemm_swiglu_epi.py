"""Cost of the SwiGLU gate inside the gate|up GEMM's epilogue (ring kernel EPI 2) against
the plain GEMM, the GEMM + one-pass gate kernel, and hipBLASLt + eager torch gate, on the
Llama-3-8B gate|up shapes (TP = 1 and the TP = 2 / 8 shards).  Median of CUDA-event
timings; one JSON line per shape.

    python benchmarks/gemm_swiglu_epi.py
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_nt, gemm_nt_swiglu, swiglu_pairs  # noqa: E402


def time_ms(fn, iters=30, warmup=5):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


for M, N, K in ((4096, 28672, 4096), (4096, 14336, 4096), (4096, 3584, 4096)):
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    glu = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    res = {
        "MxNxK": f"{M}x{N}x{K}",
        "gemm_ms": time_ms(lambda: gemm_nt(a, b, out=h)),
        "gemm_epi_gate_ms": time_ms(lambda: gemm_nt_swiglu(a, b, h, glu)),
        "gemm_plus_gate_kernel_ms": time_ms(lambda: (gemm_nt(a, b, out=h), swiglu_pairs(h, out=glu))),
        "hipblaslt_plus_eager_gate_ms": time_ms(
            lambda: (torch.matmul(a, b.t(), out=h), torch.nn.functional.silu(h[:, 0::2]) * h[:, 1::2])),
    }
    res = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}
    res["gate_cost_in_epilogue_us"] = round((res["gemm_epi_gate_ms"] - res["gemm_ms"]) * 1e3, 1)
    print(json.dumps(res), flush=True)
