"""In-kernel s_memtime stamps of the four-wave LDS-ring GEMM (diagnostic build, STAMP=1).

    python benchmarks/gemm_stamps.py M N K [SCHED_BITS]

Runs the ring kernel (gemm_w4.hip, k_gemm_w4r<.., STAMP=1>) after warm-up launches and
prints, over all waves, the median and p90 of the cycles each wave spends in the
prologue (first three K-steps in flight, step 0 read), the main loop, the epilogue, and
the phase-end waits inside the loop (s_waitcnt vmcnt(16) lgkmcnt(0) + s_barrier), plus
the loop cycles per phase against the 64 x 16 = 1024 MFMA cycles of a phase.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import _native  # noqa: E402
from collective_communication_mpi_amd.ops import gemm_nt  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
extra = int(sys.argv[4]) if len(sys.argv) > 4 else 0
D = _native.device()
a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
tiles = ((M + 255) // 256) * ((N + 255) // 256)
dbg = torch.zeros(tiles * 4 * 4, dtype=torch.int64, device="cuda")
D.gemm_set_w4_debug(dbg.data_ptr())
D.gemm_set_kernel(5)
D.gemm_set_w4_sched(8 | 512 | extra)
for _ in range(20):
    gemm_nt(a, b, out=c)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
gemm_nt(a, b, out=c)
ev1.record()
torch.cuda.synchronize()
D.gemm_set_kernel(0)
D.gemm_set_w4_sched(1)
d = dbg.view(-1, 4).double().cpu()
d = d[d[:, 1] > 0]  # a persistent grid stamps its first tile only: fewer rows than tiles
nph = K // 32


def q(col, p):
    return float(torch.quantile(d[:, col], p))


out = {"shape": [M, N, K], "ms": ev0.elapsed_time(ev1), "waves": d.shape[0], "phases": nph}
for i, name in enumerate(["prologue", "loop", "epilogue", "loop_wait"]):
    out[name] = {"p50": q(i, 0.5), "p90": q(i, 0.9)}
out["loop_cyc_per_phase_p50"] = out["loop"]["p50"] / nph
out["wait_cyc_per_phase_p50"] = out["loop_wait"]["p50"] / nph
out["mfma_frac_of_loop"] = 1024 * nph / out["loop"]["p50"]
print(json.dumps(out))
