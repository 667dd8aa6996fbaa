"""Bandwidth of the 16-bit transpose kernels on the MLP backward's operand shapes.

    python benchmarks/transpose_bench.py             # LDS-tiled kernel (default)
    CCMPI_TRANSPOSE=reg python benchmarks/transpose_bench.py

One JSON line: per shape, microseconds and the bytes moved (read + write) per second."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import transpose  # noqa: E402

out = {"kernel": os.environ.get("CCMPI_TRANSPOSE", "lds")}
for R, C in ((4096, 28672), (4096, 14336), (4096, 4096)):
    x = torch.randn(R, C, device="cuda").bfloat16()
    y = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    transpose(x, out=y)
    assert torch.equal(y, x.T)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        transpose(x, out=y)
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    out[f"{R}x{C}"] = {"us": round(us, 1), "TBps": round(4 * R * C / us / 1e6, 2)}
print(json.dumps(out), flush=True)
