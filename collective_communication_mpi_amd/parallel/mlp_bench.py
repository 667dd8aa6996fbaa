"""Tensor-parallel Llama-3-8B MLP block measurement (``ParallelSwiGLUMLP``), shared by
``benchmarks/tp_mlp.py`` and ``bench.py`` (its ``tp_mlp`` record, one TP group over all
ranks: over xGMI when each rank has its own GPU).

The block is ``y = W_down (silu(W_gate x) * W_up x)``; the gate|up GEMM carries the SwiGLU
gate in its epilogue, the down GEMM's partial output is summed by one TP all-reduce
(forward) and dX of gate|up by another (backward, overlapped with the dW GEMM).  This is
the reference's TP layer (model/func_impl.py:65-109: column-parallel projections,
row-parallel output, collective between) on a realistic shape."""
from __future__ import annotations

import statistics
import time
from typing import Dict

import torch

from . import tensor_parallel as tp
from .tensor_parallel import ParallelSwiGLUMLP, all_reduce_


def measure_tp_mlp(comm, tokens: int = 4096, d: int = 4096, ffn: int = 14336, iters: int = 10, warmup: int = 3,
                   eager_gate: bool = False, variants: bool = False, mode: str = "", modes=None) -> Dict:
    """Median forward and forward + backward times (max over ranks), the whole group's
    model TFLOP/s, the T x d bf16 TP all-reduce alone, and the host calls the device
    plane made during one steady-state forward + backward (0 expected).  ``variants``
    (p > 1): the same block with each row-parallel mode (plain / chunked / fused / push)
    side by side FIRST; the fastest correct one is recorded as this shape's ``auto`` (the
    group's ``row_modes``, CCMPI_TUNE_FILE), and the headline then runs ``auto``.
    ``modes``: the row modes of that side-by-side (default all of ``tp.ROW_MODES``).
    Collective: every rank calls."""
    from .. import mpi as MPI

    hc = comm.comm
    p = comm.Get_size()
    dev = torch.device("cuda", torch.cuda.current_device())

    def build(m):
        return ParallelSwiGLUMLP(d, ffn, comm, device=dev, dtype=torch.bfloat16, seed=1, mode=m)

    x = (torch.randn(tokens, d, generator=torch.Generator().manual_seed(3)) * 0.5).to(torch.bfloat16).to(dev)
    x.requires_grad_(True)
    gy = (torch.randn(tokens, d, generator=torch.Generator().manual_seed(4)) * 0.01).to(torch.bfloat16).to(dev)

    def timed(fn):
        # back-to-back steps between two synchronisations, as a training loop issues them
        # (the host queues step i+1 while the GPU runs step i); one synchronised call per
        # sample measured the host's launch latency too (~0.12 ms on a 1.06 ms forward,
        # profiles/r4_probe).  Median over 3 rounds of `iters` steps, max over ranks.
        for _ in range(warmup):
            fn()
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            hc.Barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / iters)
        return hc.allreduce(statistics.median(ts), op=MPI.MAX)

    def run(mlp):
        gate_up, down = mlp.gate_up, mlp.down

        def block(xx):
            if not eager_gate:
                return mlp(xx)
            h = gate_up(xx)
            return down(torch.nn.functional.silu(h[:, 0::2]) * h[:, 1::2])  # shard rows are (gate, up) pairs

        def fwd():
            with torch.no_grad():
                block(x)

        def fwd_bwd():
            x.grad = None
            gate_up.weight.grad = None
            down.weight.grad = None
            block(x).backward(gy)

        t_f = timed(fwd)
        t_fb = timed(fwd_bwd)
        host = None
        if p > 1:
            dg = comm.dev if mlp.comm is comm else tp.device_group_for(mlp.comm)
            torch.cuda.synchronize()
            h0 = dg.host_calls
            fwd_bwd()
            torch.cuda.synchronize()
            host = dg.host_calls - h0
        with torch.no_grad():  # checksum: identical across TP degrees up to bf16 rounding
            chk = float(block(x).float().abs().mean().item())
        return t_f, t_fb, host, chk

    flop_f = 2 * tokens * d * 2 * ffn + 2 * tokens * ffn * d  # whole block (all ranks together)
    var = None
    if variants and p > 1:
        # every row-parallel mode side by side, each checked against plain on the same input
        # (push / chunked sum the same partials in rank order: bitwise equal); the fastest
        # correct forward becomes this (M, N)'s "auto" for groups of this identity -- written
        # to CCMPI_TUNE_FILE like the collectives' table, and used by the headline below
        var, ref = {}, None
        for m in (modes or tp.ROW_MODES):
            rec, err, exact, close, ran_ok = None, None, 0, 0, 0
            try:
                mlp = build(m)
                vf, vfb, vh, vchk = run(mlp)
                calls0 = dict(tp.CALLS)
                with torch.no_grad():
                    out_m = mlp(x)
                ran = [k for k, v in tp.CALLS.items() if v != calls0.get(k, 0) and k.startswith("row_")]
                if ref is None:
                    ref = out_m
                exact = int(torch.equal(out_m, ref))
                close = int(torch.allclose(out_m.float(), ref.float(), rtol=2e-2, atol=2e-3))
                ran_ok = int(any(r == f"row_{m}" for r in ran))  # the mode ran (not a fallback)
                rec = {"fwd_ms": round(vf * 1e3, 3), "fwd_bwd_ms": round(vfb * 1e3, 3), "host_calls_per_step": vh,
                       "out_abs_mean": round(vchk, 6), "ran": ran}
                del mlp, out_m
            except Exception as e:  # noqa: BLE001 - one variant must not cost the record
                err = f"{type(e).__name__}: {e}"[:200]
            # every outcome agreed on every rank -- a rank that raised still makes these
            # calls, so the group's collectives stay matched and every rank sees one verdict
            ok_all = bool(hc.allreduce(int(err is None), op=MPI.MIN))
            exact = bool(hc.allreduce(exact, op=MPI.MIN))
            close = bool(hc.allreduce(close, op=MPI.MIN))
            ran_ok = bool(hc.allreduce(ran_ok, op=MPI.MIN))
            if not ok_all:
                var[m] = {"error": err or "failed on another rank"}
                continue
            var[m] = {**rec, "bitwise_equal_plain": exact, "close_to_plain": close, "ran_as_named": ran_ok}
        ok = {m: v["fwd_ms"] for m, v in var.items()
              if "error" not in v and v["close_to_plain"] and (m != "push" or v["bitwise_equal_plain"])
              and v["ran_as_named"]}
        # fwd_ms is already the max over ranks; rank 0's choice is everyone's regardless
        best = hc.bcast(min(ok, key=ok.get) if ok else None, root=0)
        if best:
            dg = comm.dev
            dg.row_modes[(tokens, d)] = best
            path = getattr(dg, "tune_file", None)
            if path and comm.Get_rank() == 0:
                from ..device import save_row_modes

                save_row_modes(path, dg.tune_key, dg.row_modes)
            hc.Barrier()
            var["auto_choice"] = best
    default_mode = tp._row_mode(mode or tp._ROW_MODE, comm, tokens, d) if p > 1 else "local"
    calls0 = dict(tp.CALLS)
    t_f, t_fb, host, chk = run(build(mode))
    paths = {k: v - calls0.get(k, 0) for k, v in tp.CALLS.items() if v != calls0.get(k, 0)}
    buf = torch.randn(tokens, d, device=dev).to(torch.bfloat16)
    t_ar = timed(lambda: all_reduce_(buf, comm)) if p > 1 else 0.0
    out = {
        "tp": p, "gate": "eager" if eager_gate else "fused", "row_mode": default_mode,
        "tokens": tokens, "d_model": d, "ffn": ffn,
        "dtype": "bf16", "shared_gpu": bool(comm.dev.shared_device) if p > 1 else False,
        "fwd_ms": round(t_f * 1e3, 3), "fwd_bwd_ms": round(t_fb * 1e3, 3),
        "fwd_TFLOPs": round(flop_f / t_f / 1e12, 1), "fwd_bwd_TFLOPs": round(3 * flop_f / t_fb / 1e12, 1),
        "tp_allreduce_bytes": tokens * d * 2, "tp_allreduce_ms": round(t_ar * 1e3, 3),
        "host_calls_per_step": host, "tp_paths": paths, "out_abs_mean": round(chk, 6)}
    if var is not None:
        out["row_mode_variants"] = var
    return out
