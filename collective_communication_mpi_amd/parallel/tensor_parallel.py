"""Megatron-style tensor-parallel layers for any torch model, on this framework's
collectives.

The reference splits ``fc_q/k/v`` by output features and ``fc_o`` by input
features (model/func_impl.py:65-70) and moves activations with its naive
collects (:76-187).  These autograd-aware modules generalise that to any
``torch.nn.Module``:

* ``ColumnParallelLinear`` -- weight rows (output features) sharded over the TP
  group; the input is replicated (backward: TP all-reduce of dX, Megatron's
  "f"); optional ``gather_output`` = the reference's forward all-gather
  (``naive_collect_forward_output``; backward = the local slice,
  ``naive_collect_backward_output``).
* ``RowParallelLinear`` -- weight columns (input features) sharded; the
  sharded input gives a partial output summed by ONE TP all-reduce (Megatron's
  "g", forward) instead of the reference's two all-gathers; with
  ``input_is_parallel=False`` the input is split here (backward: all-gather).

Collectives run on the tensors' plane: CUDA tensors use the device plane
(hand-written xGMI kernels, ``device_group_for``), CPU tensors the C++ host
plane -- the reference's own CPU/NumPy setting.  CUDA bf16 GEMMs run on the
hand-written MFMA kernels: forward ``ops.gemm_nt`` (the four-wave LDS-ring kernel
for large shapes), input gradient dX = dY W and weight gradient dW = dY^T X on the
ring kernel with K-major operands (``ops.gemm_ring``, no transposes), fp32
accumulation, bf16 out (profiles/r3_gemm: 0.95-1.04x hipBLASLt on the Llama MLP
backward shapes).  ``CCMPI_TP_GEMM=blas`` routes them to hipBLASLt instead; other
dtypes use ``torch.matmul``.
"""
from __future__ import annotations

import collections
import math
import os
from typing import Optional

import torch

from ..ops import gemm_nt, gemm_nt_swiglu, gemm_ring, gemm_tn, swiglu_pairs, swiglu_pairs_backward, transpose
from ..ops.kernels import _kmajor_via_transpose
from .layout import _host_comm, device_group_for


def _size_rank(comm):
    hc = _host_comm(comm)
    return hc.Get_size(), hc.Get_rank()


def all_reduce_(t: torch.Tensor, comm) -> torch.Tensor:
    """In-place SUM over ``comm`` of a contiguous tensor (device or host plane): ``t`` is
    overwritten with the sum (use ``all_reduce`` to keep it)."""
    p, _ = _size_rank(comm)
    if p == 1:
        return t
    if not t.is_contiguous():
        raise ValueError("all_reduce_ needs a contiguous tensor")
    if t.is_cuda:
        device_group_for(comm).allreduce(t, t, "SUM")
    else:
        from .. import mpi as MPI

        _host_comm(comm).Allreduce(MPI.IN_PLACE, t.detach().numpy(), op=MPI.SUM)
    return t


def all_reduce(t: torch.Tensor, comm) -> torch.Tensor:
    """SUM over ``comm`` into a new tensor; ``t`` is not modified (device or host plane)."""
    p, _ = _size_rank(comm)
    if p == 1:
        return t
    out = torch.empty_like(t, memory_format=torch.contiguous_format)
    if t.is_cuda:
        device_group_for(comm).allreduce(t.contiguous(), out, "SUM")
        return out
    out.copy_(t)
    return all_reduce_(out, comm)


def _gather_last(x: torch.Tensor, comm) -> torch.Tensor:
    p, _ = _size_rank(comm)
    if p == 1:
        return x
    from .layout import _dev_allgather_lastaxis, _host_allgather_lastaxis

    if x.is_cuda:
        return _dev_allgather_lastaxis(x, comm, p)
    lead = x.shape[:-1]
    x3 = x.detach().contiguous().reshape(1, -1, x.shape[-1]).numpy()
    out = _host_allgather_lastaxis(x3, comm)
    return torch.from_numpy(out).reshape(*lead, out.shape[-1])


def _slice_last(x: torch.Tensor, comm) -> torch.Tensor:
    p, r = _size_rank(comm)
    if p == 1:
        return x
    k = x.shape[-1] // p
    return x[..., r * k:(r + 1) * k].contiguous()


class _CopyToTP(torch.autograd.Function):
    """Identity forward, TP all-reduce of the gradient (Megatron "f").  Out of place: the
    incoming gradient may be aliased (e.g. handed unchanged to two branches by an add),
    so it is never modified; the reduced gradient is a fresh tensor."""

    @staticmethod
    def forward(ctx, x, comm):
        ctx.comm = comm
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return all_reduce(g, ctx.comm), None


class _ReduceFromTP(torch.autograd.Function):
    """TP all-reduce forward (out of place: the caller's tensor is not modified), identity
    backward (Megatron "g").  The TP layers themselves never go through here: their GEMMs
    write into persistent symmetric scratch that the all-reduce consumes
    (``_RowParallelFn``), which needs neither a copy nor a host call."""

    @staticmethod
    def forward(ctx, x, comm):
        return all_reduce(x, comm)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherLastTP(torch.autograd.Function):
    """Last-axis all-gather forward (reference naive_collect_forward_*), own-slice backward
    (reference naive_collect_backward_output)."""

    @staticmethod
    def forward(ctx, x, comm):
        ctx.comm = comm
        return _gather_last(x, comm)

    @staticmethod
    def backward(ctx, g):
        return _slice_last(g, ctx.comm), None


class _ScatterLastTP(torch.autograd.Function):
    """Own last-axis slice forward, all-gather backward."""

    @staticmethod
    def forward(ctx, x, comm):
        ctx.comm = comm
        return _slice_last(x, comm)

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g.contiguous(), ctx.comm), None


def copy_to_tensor_parallel_region(x, comm):
    return _CopyToTP.apply(x, comm)


def reduce_from_tensor_parallel_region(x, comm):
    return _ReduceFromTP.apply(x, comm)


def gather_from_tensor_parallel_region(x, comm):
    return _GatherLastTP.apply(x, comm)


def scatter_to_tensor_parallel_region(x, comm):
    return _ScatterLastTP.apply(x, comm)


# GEMMs of these layers: hand-written MFMA kernels (default, CCMPI_TP_GEMM=own|auto) or
# hipBLASLt (CCMPI_TP_GEMM=blas, for A/B runs).  Round 2 routed every GEMM above 2^33
# multiply-adds to hipBLASLt (our 256x256 kernel was at 0.70-0.86x on the Llama MLP
# shapes); the LDS-ring kernel closed most of that gap (profiles/r3_gemm).
_TP_GEMM = os.environ.get("CCMPI_TP_GEMM", "auto")


def _gpu_shared(comm) -> bool:
    """Whether this process shares its GPU with other ranks (multi-process-per-GPU tests):
    then the whole-CU LDS-ring GEMM must not run, since its workgroups cannot start
    beside a peer's spinning collective CTAs.  Measured by every device group (PCI bus
    ids gathered over its ranks); a size-1 group (e.g. the TP group of a pure-DP run)
    asks whether ANY group of this process found its GPU shared.  CCMPI_SHARED_RING=1
    keeps the ring (the device groups then hold every collective to half the CUs)."""
    from .. import device as _device

    if os.environ.get("CCMPI_SHARED_RING") == "1":
        return False
    if comm is None or _size_rank(comm)[0] == 1:
        return _device.SHARED_GPU_IN_PROCESS
    dg = device_group_for(comm)
    v = getattr(dg, "_tp_shared_agreed", None)
    if v is None:
        # the kernel routes this picks must be the same on every rank of the group (push vs
        # plain row mode, ring vs fallback GEMMs around a collective): the process-global part
        # differs between processes, so the group agrees once (one host all-reduce, cached)
        from .. import mpi as MPI

        local = bool(dg.shared_device) or _device.SHARED_GPU_IN_PROCESS
        v = dg._tp_shared_agreed = bool(dg.host.allreduce(int(local), op=MPI.MAX))
    return v


def _mfma_ok(x: torch.Tensor, w: torch.Tensor, comm=None) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0):
        return False
    return _TP_GEMM != "blas"


def _linear_backward(g2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, need_dx: bool, need_dw: bool,
                     comm=None, g2t: Optional[torch.Tensor] = None):
    """dX = dY W and dW = dY^T X (bf16 out, fp32 accumulate) on the LDS-ring kernel with
    K-major operands; the older routes (transpose + NT kernel, 256x256 TN kernel) when
    it does not apply (K % 64, alignment) or when the TP group's ranks share a GPU (a
    ring workgroup needs a whole CU and cannot start beside a peer's spinning
    collective CTAs: DeviceGroup disables the ring GEMMs of such a process)."""
    ring = not _gpu_shared(comm)
    dx = dw = None
    if need_dx:
        dx = gemm_ring(g2, w, False, True) if ring else None
        if dx is None:
            dx = gemm_nt(g2, transpose(w))
    if need_dw:
        dw = gemm_ring(g2, x2, True, True, a_nt=g2t) if ring else None
        if dw is None:
            dw = gemm_tn(g2, x2).to(w.dtype)
    return dx, dw


# How RowParallelLinear produces its all-reduced output (CCMPI_TP_ROW_MODE, or the layer's
# ``mode``; read at call time):
# * "plain"   -- the GEMM writes its partial product into persistent symmetric-heap
#   scratch, one two-shot all-reduce reduces it into the (ordinary, fresh) output;
# * "chunked" -- the same in CCMPI_TP_CHUNKS row blocks: block i's all-reduce runs on the
#   communication stream while block i+1's GEMM runs (no CTA spins inside a GEMM);
# * "fused"   -- the all-reduce in the GEMM epilogue (DeviceGroup.gemm_allreduce): tile
#   owners spin on peers' tiles inside the GEMM (3.1x slower at TP = 2 on a shared GPU,
#   profiles/r3_tp2).
# * "push"    -- the GEMM epilogue stores row block j of the partial straight into rank j's
#   inbox (posted writes under the GEMM, nobody spins), then one inbox-to-local two-shot
#   (DeviceGroup.gemm_push_allreduce).  Needs M % (256 p) == 0, no bias and the ring GEMM
#   (a GPU of its own, or CCMPI_SHARED_RING); otherwise plain.
# * "auto" (default) -- the mode the bench's mlp phase MEASURED fastest for this (M, N) on a
#   group of the same identity (size, GPU sharing, GPU model), read from CCMPI_TUNE_FILE
#   (``DeviceGroup.row_modes``; every rank loads the same file, so the choice is the same on
#   every rank); "plain" when nothing was measured.  "chunked" is never the unmeasured
#   default: a row block of fewer 256x256 tiles than CUs takes as long as the whole GEMM (one
#   wave either way), so at the Llama shapes (4096 x 4096 = 256 tiles, 128 per half) chunking
#   doubles the GEMM time; "push" is only chosen when it measured faster AND bitwise equal to
#   "plain" (parallel/mlp_bench.py).
ROW_MODES = ("plain", "chunked", "fused", "push")
_ROW_MODE = os.environ.get("CCMPI_TP_ROW_MODE", "auto")


def row_mode_from_table(table: dict, M: int, N: int) -> str:
    """``auto``'s choice from a measured {(M, N): mode} table (pure: tests)."""
    mode = table.get((int(M), int(N)))
    return mode if mode in ROW_MODES else "plain"


def _row_mode(mode: str, comm, M: int = 0, N: int = 0) -> str:
    """The row-parallel mode a call with a [M, N] output runs (resolves ``auto``)."""
    if mode != "auto":
        return mode
    if _size_rank(comm)[0] == 1:
        return "plain"
    return row_mode_from_table(getattr(device_group_for(comm), "row_modes", {}), M, N)


_CUS: dict = {}


def _cu_count() -> int:
    """CUs of the current device (cached per device index)."""
    try:
        idx = torch.cuda.current_device()
    except Exception:  # noqa: BLE001 - no GPU: the MI355X's
        return 256
    if idx not in _CUS:
        _CUS[idx] = int(torch.cuda.get_device_properties(idx).multi_processor_count) or 256
    return _CUS[idx]
_TP_CHUNKS = int(os.environ.get("CCMPI_TP_CHUNKS", "2"))
# which TP paths ran (tests assert the path they meant to exercise actually ran)
CALLS: "collections.Counter[str]" = collections.Counter()


def _scratch(comm, role: str, shape, dtype):
    """Persistent symmetric-heap scratch of the TP group, shared by every layer (each use
    is joined before the next layer's GEMM writes it, and a collective ends only after
    every peer read of it): one grow-only block per (role, dtype) -- a view of it for each
    shape, so varying token counts reuse it (``DeviceGroup.scratch_view``); no host call
    once it is large enough."""
    return device_group_for(comm).scratch_view("tp_" + role, shape, dtype)


def _dev_path(x2: torch.Tensor, w: torch.Tensor, comm) -> bool:
    """The hand-written device path of the TP layers: CUDA bf16 MFMA GEMMs + device TP
    collectives on a group of more than one rank (16-B aligned rows)."""
    return _mfma_ok(x2, w, comm) and _size_rank(comm)[0] > 1 and w.shape[0] % 8 == 0


def _fused_ok(x2: torch.Tensor, w: torch.Tensor, comm) -> bool:
    """The row-parallel GEMM can carry its TP all-reduce in its epilogue (DeviceGroup.
    gemm_allreduce): CUDA bf16, K shard % 64, N % 8, a group of more than one rank."""
    if not (x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    p, _ = _size_rank(comm)
    return p > 1 and x2.shape[1] % 64 == 0 and w.shape[0] % 8 == 0 and x2.shape[0] > 0


def _push_ok(x2: torch.Tensor, w: torch.Tensor, b, comm) -> bool:
    """The push row-parallel form applies (identical answer on every rank of the group):
    CUDA bf16, no bias, M % (256 p), K shard % 64, N % 8, the ring GEMM allowed."""
    if not (x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16) or b is not None:
        return False
    p, _ = _size_rank(comm)
    M, K = x2.shape
    return (p > 1 and M > 0 and M % (256 * p) == 0 and K % 64 == 0 and w.shape[0] % 8 == 0
            and x2.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and not _gpu_shared(comm))


def _chunk_rows(M: int, c: int) -> list:
    """Row blocks of the chunked row-parallel output: multiples of 256 rows (whole GEMM
    tiles), at most ``c`` of them."""
    step = max(256, -(-M // max(1, c)) // 256 * 256)
    return [(r0, min(M, r0 + step)) for r0 in range(0, M, step)]


def _deliver_wgrad(w: torch.Tensor, dw):
    """Hand a weight gradient to its DDP bucket directly when the weight has a gradient
    sink (``DistributedDataParallel(grad_sink=True)``): copied / added into the bucket view,
    the bucket notified, and None returned (autograd then has nothing to accumulate)."""
    sink = getattr(w, "_ccmpi_grad_sink", None)
    if sink is None or dw is None:
        return dw
    view, acc = sink.begin()
    if acc:
        view.add_(dw.view_as(view), alpha=sink.scale)
    elif sink.scale != 1.0:
        torch.mul(dw.view_as(view), sink.scale, out=view)
    else:
        view.copy_(dw.view_as(view))
    CALLS["wgrad_sink"] += 1
    sink.done()
    return None


def _wgrad(g2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, comm, g2t: Optional[torch.Tensor] = None):
    """dW = dY^T X.  With a DDP gradient sink on ``w`` the MFMA kernel writes (or, when
    accumulating over micro-batches, adds) straight into the bucket view: no gradient
    tensor, no AccumulateGrad pass over it (16 GB of bf16 gradients read twice and
    written once per Llama-3-8B step otherwise); returns None then."""
    sink = getattr(w, "_ccmpi_grad_sink", None)
    if sink is None or not sink.view.is_contiguous():
        return _deliver_wgrad(w, _linear_backward(g2, x2, w, False, True, comm, g2t)[1])
    view, acc = sink.begin()
    # the DDP average rides in the GEMM's alpha (sink.scale = 1/p)
    if _gpu_shared(comm) or gemm_ring(g2, x2, True, True, out=view.view(w.shape), alpha=sink.scale,
                                      accumulate=acc, a_nt=g2t) is None:
        dw = gemm_tn(g2, x2, alpha=sink.scale).to(w.dtype)
        if acc:
            view.add_(dw.view_as(view))
        else:
            view.copy_(dw.view_as(view))
    CALLS["wgrad_sink"] += 1
    sink.done()
    return None


class _RowParallelFn(torch.autograd.Function):
    """``y = sum_r x_r W_r^T (+ b)`` over the TP group (Megatron "g" folded into the layer).
    Forward on the device path: GEMM -> persistent symmetric scratch -> two-shot all-reduce
    into a fresh output (``DeviceGroup.allreduce_to_local``); the bias rides in TP rank 0's
    GEMM epilogue, so it is summed exactly once.  Backward: local (identity gradient of
    the all-reduce)."""

    @staticmethod
    def forward(ctx, x, w, b, comm, mode):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ctx.comm = comm
        ctx.save_for_backward(x2, w)
        ctx.has_bias = b is not None
        ctx.lead = x.shape[:-1]
        ctx.mfma = _mfma_ok(x2, w, comm)
        M, N = x2.shape[0], w.shape[0]
        p, r = _size_rank(comm)
        y = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
        y2 = y.view(M, N)
        if M == 0:
            return y
        if not _dev_path(x2, w, comm):
            if ctx.mfma and p == 1:
                # a one-rank TP group on the GPU: the hand-written GEMM, nothing to reduce
                CALLS["row_local"] += 1
                gemm_nt(x2, w, bias=b, out=y2)
                return y
            # host plane / other dtypes: local product, in-place all-reduce of that fresh tensor
            CALLS["row_host"] += 1
            torch.matmul(x2, w.t(), out=y2)
            all_reduce_(y2, comm)
            if b is not None:
                y2 += b
            return y
        dev = device_group_for(comm)
        bias0 = b if r == 0 else None
        mode = _row_mode(mode, comm, M, N)
        if mode == "fused" and _fused_ok(x2, w, comm):
            CALLS["row_fused"] += 1
            out = _scratch(comm, "row_fused", (M, N), torch.bfloat16)
            dev.gemm_allreduce(x2, w, bias=b, out=out)
            y2.copy_(out)
            return y
        if mode == "push" and _push_ok(x2, w, b, comm):
            CALLS["row_push"] += 1
            dev.gemm_push_allreduce(x2, w, y2)
            return y
        part = _scratch(comm, "row_partial", (M, N), x.dtype)
        blocks = _chunk_rows(M, _TP_CHUNKS) if mode == "chunked" else [(0, M)]
        if len(blocks) == 1:
            CALLS["row_plain"] += 1
            gemm_nt(x2, w, bias=bias0, out=part)
            dev.allreduce_to_local(part, y2)
            return y
        CALLS["row_chunked"] += 1
        works = []
        for r0, r1 in blocks:
            gemm_nt(x2[r0:r1], w, bias=bias0, out=part[r0:r1])
            # block i's all-reduce on the communication stream, under block i+1's GEMM
            works.append(dev.start("allreduce_to_local", part[r0:r1], y2[r0:r1]))
        for wk in works:
            wk.wait()
        return y

    @staticmethod
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1]).contiguous()
        dx = dw = db = None
        if ctx.mfma and g2.dtype == torch.bfloat16:
            if ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and _concurrent_ok(g2, ctx.comm):
                dx, dw = _concurrent_dx_dw(g2, x2, w, ctx.comm)
            else:
                dx, _ = _linear_backward(g2, x2, w, ctx.needs_input_grad[0], False, ctx.comm)
                if ctx.needs_input_grad[1]:
                    dw = _wgrad(g2, x2, w, ctx.comm)
        else:
            if ctx.needs_input_grad[0]:
                dx = g2 @ w
            if ctx.needs_input_grad[1]:
                dw = _deliver_wgrad(w, g2.t() @ x2)
        if dx is not None:
            dx = dx.reshape(*ctx.lead, w.shape[1])
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = g2.float().sum(0).to(g.dtype)
        return dx, dw, db, None, None


_SIDE_STREAMS: dict = {}


def _concurrent_ok(g2: torch.Tensor, comm) -> bool:
    """dX and dW of a row-parallel layer on two streams (CCMPI_TP_BWD_CONCURRENT, default
    on): CUDA, the ring GEMMs on (a GPU of its own, or CCMPI_SHARED_RING), no graph capture."""
    return (g2.is_cuda and os.environ.get("CCMPI_TP_BWD_CONCURRENT", "1") == "1" and not _gpu_shared(comm)
            and not torch.cuda.is_current_stream_capturing())


def _concurrent_dx_dw(g2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, comm):
    """dW = dY^T X on a second stream beside dX = dY W.  Two independent GEMMs whose last
    waves of tiles would each leave CUs idle (the Llama down projection: 896 tiles = 3.5
    waves of 256 workgroups) fill each other's tails.  A DDP gradient sink in dW records its
    bucket's ready event on that stream, so the bucket all-reduce still follows the GEMM."""
    cur = torch.cuda.current_stream(g2.device)
    side = _SIDE_STREAMS.get(g2.device)
    if side is None:
        side = _SIDE_STREAMS[g2.device] = torch.cuda.Stream(device=g2.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        dw = _wgrad(g2, x2, w, comm)
    dx, _ = _linear_backward(g2, x2, w, True, False, comm)
    cur.wait_stream(side)
    if dw is not None:
        dw.record_stream(cur)
    CALLS["row_bwd_concurrent"] += 1
    return dx, dw


def _column_backward(g2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, need_dx: bool, need_dw: bool, comm,
                     g2t: Optional[torch.Tensor] = None):
    """Backward of a column-parallel projection with its TP all-reduce of dX (Megatron "f")
    overlapped with the weight-gradient GEMM: dX's partial product goes into persistent
    symmetric scratch, its all-reduce into a fresh dX starts on the communication stream,
    and dW = dY^T X runs on the compute stream meanwhile."""
    if not (need_dx and _dev_path(g2, w, comm)):
        dx, _ = _linear_backward(g2, x2, w, need_dx, False, comm)
        if dx is not None:
            dx = all_reduce_(dx, comm)  # a fresh tensor of this backward: in place is safe
        return dx, (_wgrad(g2, x2, w, comm, g2t) if need_dw else None)
    CALLS["col_bwd_overlap"] += 1
    dev = device_group_for(comm)
    M, K = g2.shape[0], w.shape[1]
    part = _scratch(comm, "dx_partial", (M, K), g2.dtype)
    ring = not _gpu_shared(comm)
    if not (ring and gemm_ring(g2, w, False, True, out=part) is not None):
        gemm_nt(g2, transpose(w), out=part)
    dx = torch.empty(M, K, device=g2.device, dtype=g2.dtype)
    work = dev.start("allreduce_to_local", part, dx)
    dw = _wgrad(g2, x2, w, comm, g2t) if need_dw else None
    work.wait()
    return dx, dw


class _ColumnParallelFn(torch.autograd.Function):
    """``y = x W_r^T (+ b_r)`` with the replicated input's gradient all-reduced over the TP
    group in the backward, overlapped with the dW GEMM (``_column_backward``)."""

    @staticmethod
    def forward(ctx, x, w, b, comm):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ctx.comm = comm
        ctx.save_for_backward(x2, w)
        ctx.has_bias = b is not None
        ctx.lead = x.shape[:-1]
        ctx.mfma = _mfma_ok(x2, w, comm)
        y = torch.empty(*x.shape[:-1], w.shape[0], device=x.device, dtype=x.dtype)
        y2 = y.view(-1, w.shape[0])
        if ctx.mfma:
            gemm_nt(x2, w, bias=b, out=y2)
        else:
            torch.matmul(x2, w.t(), out=y2)
            if b is not None:
                y2 += b
        return y

    @staticmethod
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1]).contiguous()
        dx = dw = db = None
        if ctx.mfma and g2.dtype == torch.bfloat16:
            dx, dw = _column_backward(g2, x2, w, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.comm)
        else:
            if ctx.needs_input_grad[1]:
                dw = _deliver_wgrad(w, g2.t() @ x2)
            if ctx.needs_input_grad[0]:
                dx = all_reduce_(g2 @ w, ctx.comm)
        if dx is not None:
            dx = dx.reshape(*ctx.lead, w.shape[1])
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = g2.float().sum(0).to(g.dtype)
        return dx, dw, db, None


def _bind_device_group(comm, device) -> None:
    """Collective, at construction (every rank builds the same layers): create the TP group's
    device plane before the first GEMM, so a process that shares its GPU with other ranks
    has switched its GEMMs off the whole-CU ring kernel (DeviceGroup) before any runs."""
    if device is None or torch.device(device).type != "cuda":
        return
    if _size_rank(comm)[0] > 1:
        device_group_for(comm)


def _init_full(out_f: int, in_f: int, seed: int, dtype, bias: bool, device=None):
    """Full (unsharded) weights from a seeded generator: identical on every rank.  On the
    CPU by default (tests regenerate them there); ``device`` (CUDA) draws them on the GPU
    instead -- same values on every rank of one GPU model, and seconds instead of minutes
    for a Llama-3-8B-sized stack."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    gen = torch.Generator(device=dev).manual_seed(seed)
    bound = 1.0 / math.sqrt(in_f)
    w = (torch.rand(out_f, in_f, generator=gen, device=dev) * 2 - 1) * bound
    b = (torch.rand(out_f, generator=gen, device=dev) * 2 - 1) * bound if bias else None
    return w.to(dtype), (b.to(dtype) if b is not None else None)


class ColumnParallelLinear(torch.nn.Module):
    """``y = x W^T + b`` with W's rows (output features) sharded over ``comm`` (TP group).

    ``gather_output=False`` returns this rank's ``out_features / p`` columns
    (feed a ``RowParallelLinear``); ``True`` all-gathers the full output."""

    def __init__(self, in_features: int, out_features: int, comm, bias: bool = True, gather_output: bool = False,
                 device=None, dtype=torch.float32, seed: int = 0, init: str = "cpu"):
        super().__init__()
        p, r = _size_rank(comm)
        if out_features % p:
            raise ValueError(f"out_features {out_features} not divisible by TP size {p}")
        self.comm, self.p, self.r = comm, p, r
        self.in_features, self.out_features = in_features, out_features
        self.gather_output = gather_output
        k = out_features // p
        _bind_device_group(comm, device)
        w, b = _init_full(out_features, in_features, seed, dtype, bias, device if init == "device" else None)
        self.weight = torch.nn.Parameter(w[r * k:(r + 1) * k].contiguous().to(device))
        self.bias = torch.nn.Parameter(b[r * k:(r + 1) * k].contiguous().to(device)) if bias else None

    def forward(self, x):
        y = _ColumnParallelFn.apply(x, self.weight, self.bias, self.comm)
        return gather_from_tensor_parallel_region(y, self.comm) if self.gather_output else y


class RowParallelLinear(torch.nn.Module):
    """``y = x W^T + b`` with W's columns (input features) sharded over ``comm``.

    The partial products are summed by one TP all-reduce; the bias is added once,
    after the reduction.  ``input_is_parallel=False`` splits a full input here."""

    def __init__(self, in_features: int, out_features: int, comm, bias: bool = True, input_is_parallel: bool = True,
                 device=None, dtype=torch.float32, seed: int = 0, mode: str = "", init: str = "cpu"):
        super().__init__()
        p, r = _size_rank(comm)
        if in_features % p:
            raise ValueError(f"in_features {in_features} not divisible by TP size {p}")
        if mode and mode not in ROW_MODES + ("auto",):
            raise ValueError(f"RowParallelLinear mode {mode!r} not in {ROW_MODES + ('auto',)}")
        self.mode = mode  # "" = CCMPI_TP_ROW_MODE at call time
        self.comm, self.p, self.r = comm, p, r
        self.in_features, self.out_features = in_features, out_features
        self.input_is_parallel = input_is_parallel
        k = in_features // p
        _bind_device_group(comm, device)
        w, b = _init_full(out_features, in_features, seed, dtype, bias, device if init == "device" else None)
        self.weight = torch.nn.Parameter(w[:, r * k:(r + 1) * k].contiguous().to(device))
        self.bias = torch.nn.Parameter(b.to(device)) if bias else None

    def forward(self, x):
        if not self.input_is_parallel:
            x = scatter_to_tensor_parallel_region(x, self.comm)
        return _RowParallelFn.apply(x, self.weight, self.bias, self.comm, self.mode or _ROW_MODE)


def _dh_transposed(h: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, comm) -> bool:
    """Whether the gate|up weight gradient dW = dh^T X takes the transposed route (then the
    SwiGLU backward also writes dh^T): the ring is on, and ops' K-major routing rule holds."""
    T, n = h.shape
    return (T % 8 == 0 and not _gpu_shared(comm) and h.stride(1) == 1
            and _kmajor_via_transpose(n, x2.shape[1], T, h, x2))


class _GateUpSwiGLU(torch.autograd.Function):
    """``a = swiglu_pairs(x W^T)`` for a column-parallel gate|up weight whose rows are
    interleaved (gate j, up j) pairs.  Forward: one GEMM whose epilogue also writes the
    gate (LDS-ring kernel, EPI 2), else GEMM + ``swiglu_pairs``; saves x, W and the GEMM
    output h.  Backward: ``swiglu_pairs_backward`` (one kernel), then dX with its TP
    all-reduce overlapped with the dW GEMM (``_column_backward``, Megatron "f")."""

    @staticmethod
    def forward(ctx, x, w, comm):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M, N = x2.shape[0], w.shape[0]
        h = torch.empty(M, N, device=x.device, dtype=x.dtype)
        a = torch.empty(*x.shape[:-1], N // 2, device=x.device, dtype=x.dtype)
        a2 = a.view(M, N // 2)
        ctx.mfma = _mfma_ok(x2, w, comm)  # False: hipBLASLt GEMMs (CCMPI_TP_GEMM=blas A/B runs)
        fused = ctx.mfma and M > 0 and not _gpu_shared(comm) and gemm_nt_swiglu(x2, w, h, a2)
        if not fused:
            if ctx.mfma:
                gemm_nt(x2, w, out=h)
            else:
                torch.matmul(x2, w.t(), out=h)
            swiglu_pairs(h, out=a2)
        ctx.comm = comm
        ctx.lead = x.shape[:-1]
        ctx.save_for_backward(x2, w, h)
        return a

    @staticmethod
    def backward(ctx, da):
        x2, w, h = ctx.saved_tensors
        da2 = da.reshape(-1, da.shape[-1])
        dht = None
        if ctx.mfma and ctx.needs_input_grad[1] and _dh_transposed(h, x2, w, ctx.comm):
            # dh^T from the same kernel: dW = dh^T X on the N-layout pair ring, no transpose pass
            dh, dht = swiglu_pairs_backward(h, da2, transposed=True)
            CALLS["dh_transposed"] += 1
        else:
            dh = swiglu_pairs_backward(h, da2)
        if ctx.mfma:
            dx, dw = _column_backward(dh, x2, w, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.comm, dht)
        else:
            dw = _deliver_wgrad(w, dh.t() @ x2) if ctx.needs_input_grad[1] else None
            dx = all_reduce_(dh @ w, ctx.comm) if ctx.needs_input_grad[0] else None
        if dx is not None:
            dx = dx.reshape(*ctx.lead, w.shape[1])
        return dx, dw, None


class ParallelSwiGLUMLP(torch.nn.Module):
    """Llama MLP block ``y = W_down (silu(W_gate x) * W_up x)`` over a TP group.

    ``gate_up`` is one ``ColumnParallelLinear`` whose rank-r shard holds the gate and up
    features ``[r k, (r+1) k)`` (k = ffn / p) as interleaved rows (gate j, up j), so the
    SwiGLU gate is local and, on CUDA bf16, applied by the gate|up GEMM's own epilogue
    (``ops.gemm_nt_swiglu``; backward one ``swiglu_pairs_backward`` kernel).  ``down`` is
    a ``RowParallelLinear`` over those k features: one TP all-reduce in forward (Megatron
    "g"), one in backward for dX of ``gate_up`` (Megatron "f").  The reference's TP layer
    (model/func_impl.py:65-109) on a realistic Llama-3-8B shape."""

    def __init__(self, d_model: int, ffn: int, comm, device=None, dtype=torch.bfloat16, seed: int = 0,
                 mode: str = "", init: str = "cpu"):
        super().__init__()
        p, r = _size_rank(comm)
        if ffn % p:
            raise ValueError(f"ffn {ffn} not divisible by TP size {p}")
        k = ffn // p
        self.comm, self.p, self.r, self.ffn = comm, p, r, ffn
        self.gate_up = ColumnParallelLinear(d_model, 2 * ffn, comm, bias=False, device=device, dtype=dtype, seed=seed,
                                            init=init)
        full, _ = _init_full(2 * ffn, d_model, seed, dtype, False, device if init == "device" else None)
        with torch.no_grad():  # shard rows: gate r k + j at 2 j, up r k + j at 2 j + 1
            shard = torch.stack([full[r * k:(r + 1) * k], full[ffn + r * k:ffn + (r + 1) * k]], dim=1)
            self.gate_up.weight.copy_(shard.reshape(2 * k, d_model))
        self.down = RowParallelLinear(ffn, d_model, comm, bias=False, device=device, dtype=dtype, seed=seed + 1,
                                      mode=mode, init=init)

    def _fused_ok(self, x) -> bool:
        w = self.gate_up.weight
        return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
                and (w.shape[0] // 2) % 4 == 0)

    def forward(self, x):
        if self._fused_ok(x):
            a = _GateUpSwiGLU.apply(x, self.gate_up.weight, self.comm)
        else:
            h = self.gate_up(x)
            a = torch.nn.functional.silu(h[..., 0::2]) * h[..., 1::2]
        return self.down(a)


def full_weight(layer, comm) -> torch.Tensor:
    """Reassemble the unsharded weight of a Column/RowParallelLinear (collective)."""
    w = layer.weight.detach()
    dim = 0 if isinstance(layer, ColumnParallelLinear) else 1
    parts = _host_comm(comm).allgather(w.float().cpu())
    return torch.cat(parts, dim=dim)


def sharded_grad_full(layer, comm) -> torch.Tensor:
    """Reassemble the unsharded weight gradient (collective), for checks."""
    g = layer.weight.grad.detach()
    dim = 0 if isinstance(layer, ColumnParallelLinear) else 1
    parts = _host_comm(comm).allgather(g.float().cpu())
    return torch.cat(parts, dim=dim)


__all__ = ["ColumnParallelLinear", "RowParallelLinear", "ParallelSwiGLUMLP", "all_reduce", "all_reduce_",
           "copy_to_tensor_parallel_region", "ROW_MODES",
           "reduce_from_tensor_parallel_region", "gather_from_tensor_parallel_region",
           "scatter_to_tensor_parallel_region", "full_weight", "sharded_grad_full"]
