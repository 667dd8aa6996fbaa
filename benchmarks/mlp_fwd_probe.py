"""Where the TP=1 MLP forward's time goes: each forward GEMM timed alone on the block's own
tensors and on uniform-random operands of the same shapes, ours and hipBLASLt, interleaved
(median of rounds).  Separates "slower in the block" effects (operand values, the previous
kernel's state) from the kernels' own speed.  One JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt, gemm_nt_swiglu  # noqa: E402
from collective_communication_mpi_amd.parallel.tensor_parallel import ParallelSwiGLUMLP  # noqa: E402


def t_ms(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


comm = Communicator(MPI.COMM_WORLD)
T, d, f = 4096, 4096, 14336
mlp = ParallelSwiGLUMLP(d, f, comm, device="cuda", dtype=torch.bfloat16, seed=1, init="device")
x = (torch.randn(T, d, device="cuda") * 0.5).bfloat16()
wgu, wd = mlp.gate_up.weight.detach(), mlp.down.weight.detach()
h = torch.empty(T, 2 * f, device="cuda", dtype=torch.bfloat16)
a = torch.empty(T, f, device="cuda", dtype=torch.bfloat16)
y = torch.empty(T, d, device="cuda", dtype=torch.bfloat16)
gemm_nt_swiglu(x, wgu, h, a)
ur = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
xr, wgur, ar, wdr = ur(T, d), ur(2 * f, d), ur(T, f), ur(d, f)
cases = {
    "forward_block": lambda: mlp(x),
    "gate_up_epi2_block": lambda: gemm_nt_swiglu(x, wgu, h, a),
    "gate_up_epi2_uniform": lambda: gemm_nt_swiglu(xr, wgur, h, a),
    "gate_up_plain_block": lambda: gemm_nt(x, wgu, out=h),
    "down_block": lambda: gemm_nt(a, wd, out=y),
    "down_uniform": lambda: gemm_nt(ar, wdr, out=y),
    "down_block_hipblaslt": lambda: torch.matmul(a, wd.T, out=y),
    "down_uniform_hipblaslt": lambda: torch.matmul(ar, wdr.T, out=y),
    "gate_up_block_hipblaslt": lambda: torch.matmul(x, wgu.T, out=h),
}
res = {k: [] for k in cases}
with torch.no_grad():
    for _ in range(5):
        for k, fn in cases.items():
            res[k].append(t_ms(fn))
out = {k: round(statistics.median(v), 4) for k, v in res.items()}
out["abs_mean"] = {"x": round(x.float().abs().mean().item(), 4), "w_gate_up": round(wgu.float().abs().mean().item(), 5),
                   "glu": round(a.float().abs().mean().item(), 5), "w_down": round(wd.float().abs().mean().item(), 5)}
print(json.dumps(out), flush=True)
