"""Split-K sweep of the small weight-gradient contractions of the harness backward:
A = dQKV^T . Xp (32768 x 768 by 32768 x 72, Xp strided inside the [h | xp] rows) and
dW_o = dZ^T . pool (2048 x 16 by 2048 x 256), atomics vs workspace + reduction."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_tn  # noqa: E402


def t(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best


def case(name, a, b, splits, accumulate):
    ref = a.float().t() @ b.float()
    out = torch.zeros(a.shape[1], b.shape[1], device="cuda")
    line = []
    for ws in (False, True):
        for sk in splits:
            out.zero_()
            gemm_tn(a, b, out=out, splitk=sk, workspace=ws)
            err = ((out - ref).norm() / ref.norm()).item()
            assert err < 1e-2, (name, sk, ws, err)
            us = t(lambda: gemm_tn(a, b, out=out, splitk=sk, workspace=ws, accumulate=accumulate))
            line.append(f"{'ws' if ws else 'at'}{sk}:{us:.1f}")
    us = t(lambda: torch.mm(a.t(), b, out=torch.empty(a.shape[1], b.shape[1], device="cuda", dtype=torch.bfloat16)))
    line.append(f"hipblaslt(bf16 out):{us:.1f}")
    print(f"{name}: " + "  ".join(line), flush=True)


M, d, kp = 32768, 768, 72
hx = torch.randn(M, 896, device="cuda").bfloat16()
xp = hx[:, d:d + kp]
dqkv = torch.randn(M, 768, device="cuda").bfloat16()
case("A=dQKV^T.Xp 768x72 K=32768", dqkv, xp, (16, 32, 64, 128, 256), False)
dz = torch.randn(2048, 16, device="cuda").bfloat16()
pool = torch.randn(2048, 256, device="cuda").bfloat16()
case("dW_o=dZ^T.pool 16x256 K=2048", dz, pool, (1, 2, 4, 8, 16, 32), True)
