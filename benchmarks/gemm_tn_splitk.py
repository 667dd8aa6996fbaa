"""Split-K sweep of the weight-gradient TN GEMM on the harness shapes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_tn  # noqa: E402
from collective_communication_mpi_amd.ops.kernels import set_tn_variant  # noqa: E402


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for M, N1, N2 in [(32768, 768, 768), (32768, 768, 72), (32768, 384, 768), (32768, 768, 384), (16384, 4096, 4096),
                  (8192, 4096, 14336)]:
    a = torch.randn(M, N1, device="cuda").bfloat16()
    b = torch.randn(M, N2, device="cuda").bfloat16()
    out = torch.empty(N1, N2, device="cuda")
    res = {}
    for variant in (0, 1):
        set_tn_variant(variant)
        res[f"v{variant}auto"] = min(t(lambda: gemm_tn(a, b, out=out)) for _ in range(3))
    set_tn_variant(1)
    for sk in (8, 16, 24, 28, 32, 48):
        if N1 >= 256 and N2 >= 256:
            res[f"v1/{sk}"] = min(t(lambda: gemm_tn(a, b, out=out, splitk=sk)) for _ in range(3))
    set_tn_variant(0)
    for sk in (None, 1, 2, 4, 8, 14, 16, 24, 32, 48, 64, 96, 128):
        if sk is not None and sk > M // 64:
            continue
        res[sk] = min(t(lambda: gemm_tn(a, b, out=out, splitk=sk)) for _ in range(3))
    set_tn_variant(None)
    best = min((v, str(k)) for k, v in res.items() if k is not None)
    print(f"{M}x{N1}x{N2}: auto(v0) {res[None]:.1f}us  best {best[1]} {best[0]:.1f}us  | " +
          " ".join(f"{k}:{v:.1f}" for k, v in res.items() if k is not None), flush=True)
