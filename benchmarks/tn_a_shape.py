"""The harness backward's A = dQKV^T Xp (32768 x 768 by 32768 x 72, fp32 atomics into A) alone,
N launches, for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_tn  # noqa: E402

dq = torch.randn(32768, 768, device="cuda").bfloat16()
xp = torch.randn(32768, 72, device="cuda").bfloat16()
a = torch.zeros(768, 72, device="cuda")
for _ in range(int(os.environ.get("N", "50"))):
    gemm_tn(dq, xp, out=a, accumulate=True, workspace=False)
torch.cuda.synchronize()
print("ok", flush=True)
