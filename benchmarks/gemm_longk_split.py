"""Long-K NT GEMM (Llama gate|up dX shape, 4096 x 4096 x 28672: 256 tiles, one per CU)
routes, interleaved rounds, median; vs fp32 reference.

* auto: gemm_nt's choice (the 256x256 ping-pong kernel for long K);
* pair: the pair-slot ring over the whole K;
* split2_fp32: two K halves on the pair ring into an fp32 workspace (second accumulates),
  then one cast to bf16;
* split2_bf16: the same accumulating straight into the bf16 output (one extra rounding);
* tb_ring: the dX = dY W form (K-major B, [K][N]) on the pair ring;
* hipblaslt.
(profiles/r4_longk: the K halves are slower than one pass; the route was not kept.)
One JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import gemm_nt, gemm_ring  # noqa: E402


def t_ms(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


M = N = 4096
K = int(os.environ.get("LONGK", "28672"))
K2 = K // 2
a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
ws = torch.empty(M, N, device="cuda")
ref = a.float() @ b.float().T


def split_fp32():
    gemm_ring(a[:, :K2], b[:, :K2], False, False, out=ws)
    gemm_ring(a[:, K2:], b[:, K2:], False, False, out=ws, accumulate=True)
    c.copy_(ws)


def split_bf16():
    gemm_ring(a[:, :K2], b[:, :K2], False, False, out=c)
    gemm_ring(a[:, K2:], b[:, K2:], False, False, out=c, accumulate=True)


# dX = dY W form (K-major B, [K][N]): the gate|up backward's long-K GEMM
bt = b.T.contiguous()


cases = {"auto": lambda: gemm_nt(a, b, out=c), "pair": lambda: gemm_ring(a, b, False, False, out=c),
         "split2_fp32": split_fp32, "split2_bf16": split_bf16,
         "tb_ring": lambda: gemm_ring(a, bt, False, True, out=c),
         "hipblaslt": lambda: torch.matmul(a, b.T, out=c)}
res, err = {k: [] for k in cases}, {}
for _ in range(5):
    for k, fn in cases.items():
        res[k].append(t_ms(fn))
        err[k] = float(((c.float() - ref).abs().max() / ref.abs().max()).item())
out = {"shape": f"{M}x{N}x{K}"}
for k, v in res.items():
    ms = statistics.median(v)
    out[k] = {"ms": round(ms, 4), "TF": round(2 * M * N * K / ms / 1e9, 1), "max_rel_err": round(err[k], 5)}
print(json.dumps(out), flush=True)
