"""Embedding/QKV weight-gradient kernel (csrc/device/wgrad.hip) at the harness shape
vs the two library sgemms it replaces: Gq only, Gq + Ge, Gq + Ge + zeroing."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402

D = _native.device()


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


R, d, kp = 768, 768, 72
A, We, Wq = (torch.randn(*sh, device="cuda") for sh in ((R, kp), (d, kp), (R, d)))
Gq, Ge, Z = torch.zeros(R, d, device="cuda"), torch.zeros(d, kp, device="cuda"), torch.zeros(R, kp, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def k(ge, z):
    D.emb_qkv_wgrad(A.data_ptr(), kp, We.data_ptr(), kp, Wq.data_ptr(), d, Gq.data_ptr(), d,
                    Ge.data_ptr() if ge else 0, kp, Z.data_ptr() if z else 0, kp, R, d, kp, st)


print(f"Gq only {t(lambda: k(False, False)):.1f} us   Gq+Ge {t(lambda: k(True, False)):.1f} us   "
      f"Gq+Ge+Z {t(lambda: k(True, True)):.1f} us", flush=True)
print(f"library: Gq.addmm_ {t(lambda: Gq.addmm_(A, We.t())):.1f} us   Ge.addmm_ {t(lambda: Ge.addmm_(Wq.t(), A)):.1f} us   "
      f"Z.zero_ {t(lambda: Z.zero_()):.1f} us", flush=True)
Ge.zero_()
k(True, True)
torch.cuda.synchronize()
print("check", ((Ge - Wq.t() @ A).abs().max() / (Wq.t() @ A).abs().max()).item())
