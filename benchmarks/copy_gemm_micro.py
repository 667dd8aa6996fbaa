"""Single-GPU micro-benchmarks: device copy (k_copy vs runtime blit) and the
MFMA GEMM vs hipBLASLt (torch.matmul) on the harness shapes + 4096^3/8192^3."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402


def tmin(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


D = _native.device()
dc = D.DeviceComm(0, 1, 0)
n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda").random_()
y = torch.empty_like(x)
st = torch.cuda.current_stream().cuda_stream
for eng in (False, True):
    dc.set_copy_engine(eng)
    ms = tmin(lambda: dc.allreduce(x.data_ptr(), y.data_ptr(), n // 4, 10, 0, 1, st, 256, False))
    print(f"copy 1GiB {'blit' if eng else 'k_copy'}: {ms:.3f} ms = {n / ms / 1e6:.0f} GB/s algbw", flush=True)
assert torch.equal(x, y)
from collective_communication_mpi_amd.ops import gemm_tn  # noqa: E402

for (M, N, K) in [(32768, 768, 72), (32768, 768, 768), (32768, 384, 768), (2048, 16, 128), (4096, 4096, 4096),
                  (8192, 8192, 8192)]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
    fl = 2 * M * N * K
    res = {}
    for glds in (False, True):
        D.gemm_set_glds(glds)
        res[glds] = tmin(lambda: gemm_nt(a, b))
    ref = tmin(lambda: a @ b.T)
    print(f"gemm_nt {M}x{N}x{K}: regstage {res[False]:.3f} ms ({fl / res[False] / 1e9:.0f} TF/s)  "
          f"glds {res[True]:.3f} ms ({fl / res[True] / 1e9:.0f} TF/s)  hipBLASLt {ref:.3f} ms ({fl / ref / 1e9:.0f} TF/s)",
          flush=True)
for (M, N1, N2) in [(32768, 384, 768), (32768, 768, 72), (4096, 4096, 4096), (4096, 14336, 4096)]:
    a = torch.randn(M, N1, device="cuda").bfloat16()
    b = torch.randn(M, N2, device="cuda").bfloat16()
    fl = 2 * M * N1 * N2
    ours = tmin(lambda: gemm_tn(a, b))
    ref = tmin(lambda: a.T @ b)
    print(f"gemm_tn {M}x{N1}x{N2}: ours {ours:.3f} ms ({fl / ours / 1e9:.0f} TF/s)  hipBLASLt {ref:.3f} ms "
          f"({fl / ref / 1e9:.0f} TF/s)", flush=True)
