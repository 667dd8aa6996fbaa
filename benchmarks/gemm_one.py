"""Run one GEMM shape/kernel repeatedly (for rocprofv3 counter collection).

    python benchmarks/gemm_one.py M N K MODE ITERS     (MODE: 0 auto, 1 128x128, 2 256x256, 3 256x128,
                                                       5 four-wave 256x256 (CCMPI_W4_SCHED), -1 hipBLASLt)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

M, N, K, mode, iters = (int(v) for v in sys.argv[1:6])
a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
if os.environ.get("CCMPI_RING_SCHED"):
    _native.device().gemm_set_ring_sched(int(os.environ["CCMPI_RING_SCHED"]))
if mode >= 0:
    _native.device().gemm_set_kernel(mode)
    if mode == 5 and os.environ.get("CCMPI_W4_SCHED"):
        _native.device().gemm_set_w4_sched(int(os.environ["CCMPI_W4_SCHED"]))
for _ in range(iters):
    if mode >= 0:
        gemm_nt(a, b, out=c)
    else:
        torch.matmul(a, b.T, out=c)
torch.cuda.synchronize()
print("done", M, N, K, mode)
