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

import math
import os

import torch

from ..ops import gemm_nt, gemm_nt_swiglu, gemm_ring, gemm_tn, swiglu_pairs, swiglu_pairs_backward, transpose
from .layout import _host_comm, device_group_for


def _size_rank(comm):
    hc = _host_comm(comm)
    return hc.Get_size(), hc.Get_rank()


def all_reduce_(t: torch.Tensor, comm) -> torch.Tensor:
    """In-place SUM over ``comm`` of a contiguous tensor (device or host plane)."""
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
    """Identity forward, TP all-reduce of the gradient (Megatron "f").  The gradient
    is reduced in place: autograd hands this node a buffer it owns, and the device
    plane registers it on demand (no copy in or out, DeviceGroup._register_call)."""

    @staticmethod
    def forward(ctx, x, comm):
        ctx.comm = comm
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return all_reduce_(g.contiguous(), ctx.comm), None


class _ReduceFromTP(torch.autograd.Function):
    """TP all-reduce forward, identity backward (Megatron "g").  The partial product
    is reduced in place (it is the fresh output of the row-parallel GEMM, which its
    backward does not need), so the 32 MiB Llama activation is never cloned."""

    @staticmethod
    def forward(ctx, x, comm):
        if not x.is_contiguous():
            return all_reduce_(x.contiguous(), comm)
        ctx.mark_dirty(x)
        return all_reduce_(x, comm)

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
    """Whether this TP group's ranks share a GPU: measured by the group itself (PCI bus
    ids gathered over the ranks, DeviceGroup.shared_device), per group."""
    if comm is None:
        return False
    return bool(device_group_for(comm).shared_device)


def _mfma_ok(x: torch.Tensor, w: torch.Tensor, comm=None) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0):
        return False
    return _TP_GEMM != "blas"


def _linear_backward(g2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, need_dx: bool, need_dw: bool,
                     comm=None):
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
        dw = gemm_ring(g2, x2, True, True) if ring else None
        if dw is None:
            dw = gemm_tn(g2, x2).to(w.dtype)
    return dx, dw


class _LinearFn(torch.autograd.Function):
    """y = x W^T (+ b): MFMA bf16 kernels on CUDA bf16, torch.matmul otherwise."""

    @staticmethod
    def forward(ctx, x, w, b, comm=None):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ctx.comm = comm
        ctx.save_for_backward(x2, w)
        ctx.has_bias = b is not None
        ctx.lead = x.shape[:-1]
        ctx.mfma = _mfma_ok(x2, w, comm)
        # the output is allocated in its final shape and written through a 2-D view, so
        # the returned tensor is no view: _ReduceFromTP may reduce it in place (mark_dirty)
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
            dx, dw = _linear_backward(g2, x2, w, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.comm)
        else:
            if ctx.needs_input_grad[0]:
                dx = g2 @ w
            if ctx.needs_input_grad[1]:
                dw = g2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = g2.float().sum(0).to(g.dtype)
        if dx is not None:
            dx = dx.reshape(*ctx.lead, w.shape[1])
        return dx, dw, db, None


# The row-parallel GEMM with its TP all-reduce fused into the epilogue (DeviceGroup.
# gemm_allreduce) is opt-in: at TP = 2 on one shared GPU the Llama MLP forward took
# 5.1 ms fused against 1.64 ms for GEMM + zero-copy all-reduce (profiles/r3_tp2); over
# xGMI it is unmeasured.
_TP_FUSED = os.environ.get("CCMPI_TP_FUSED", "0") == "1"


def _fused_ok(x2: torch.Tensor, w: torch.Tensor, comm) -> bool:
    """The row-parallel GEMM can carry its TP all-reduce in its epilogue (DeviceGroup.
    gemm_allreduce): CUDA bf16, K shard % 64, N % 8, a group of more than one rank."""
    if not (_TP_FUSED and x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    p, _ = _size_rank(comm)
    return p > 1 and x2.shape[1] % 64 == 0 and w.shape[0] % 8 == 0 and x2.shape[0] > 0


class _RowParallelFused(torch.autograd.Function):
    """y = sum_r x_r W_r^T + b with the all-reduce fused into the GEMM (forward); the
    backward is local, as for Megatron's "g" (identity gradient of the all-reduce)."""

    @staticmethod
    def forward(ctx, x, w, b, comm):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ctx.comm = comm
        ctx.save_for_backward(x2, w)
        ctx.has_bias = b is not None
        ctx.lead = x.shape[:-1]
        y = device_group_for(comm).gemm_allreduce(x2, w, bias=b)
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1]).contiguous()
        dx = dw = db = None
        dx, dw = _linear_backward(g2, x2, w, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.comm)
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


def _init_full(out_f: int, in_f: int, seed: int, dtype, bias: bool):
    """Full (unsharded) weights from a seeded CPU generator: identical on every rank."""
    gen = torch.Generator().manual_seed(seed)
    bound = 1.0 / math.sqrt(in_f)
    w = (torch.rand(out_f, in_f, generator=gen) * 2 - 1) * bound
    b = (torch.rand(out_f, generator=gen) * 2 - 1) * bound if bias else None
    return w.to(dtype), (b.to(dtype) if b is not None else None)


class ColumnParallelLinear(torch.nn.Module):
    """``y = x W^T + b`` with W's rows (output features) sharded over ``comm`` (TP group).

    ``gather_output=False`` returns this rank's ``out_features / p`` columns
    (feed a ``RowParallelLinear``); ``True`` all-gathers the full output."""

    def __init__(self, in_features: int, out_features: int, comm, bias: bool = True, gather_output: bool = False,
                 device=None, dtype=torch.float32, seed: int = 0):
        super().__init__()
        p, r = _size_rank(comm)
        if out_features % p:
            raise ValueError(f"out_features {out_features} not divisible by TP size {p}")
        self.comm, self.p, self.r = comm, p, r
        self.in_features, self.out_features = in_features, out_features
        self.gather_output = gather_output
        k = out_features // p
        _bind_device_group(comm, device)
        w, b = _init_full(out_features, in_features, seed, dtype, bias)
        self.weight = torch.nn.Parameter(w[r * k:(r + 1) * k].contiguous().to(device))
        self.bias = torch.nn.Parameter(b[r * k:(r + 1) * k].contiguous().to(device)) if bias else None

    def forward(self, x):
        x = copy_to_tensor_parallel_region(x, self.comm)
        y = _LinearFn.apply(x, self.weight, self.bias, self.comm)
        return gather_from_tensor_parallel_region(y, self.comm) if self.gather_output else y


class RowParallelLinear(torch.nn.Module):
    """``y = x W^T + b`` with W's columns (input features) sharded over ``comm``.

    The partial products are summed by one TP all-reduce; the bias is added once,
    after the reduction.  ``input_is_parallel=False`` splits a full input here."""

    def __init__(self, in_features: int, out_features: int, comm, bias: bool = True, input_is_parallel: bool = True,
                 device=None, dtype=torch.float32, seed: int = 0):
        super().__init__()
        p, r = _size_rank(comm)
        if in_features % p:
            raise ValueError(f"in_features {in_features} not divisible by TP size {p}")
        self.comm, self.p, self.r = comm, p, r
        self.in_features, self.out_features = in_features, out_features
        self.input_is_parallel = input_is_parallel
        k = in_features // p
        _bind_device_group(comm, device)
        w, b = _init_full(out_features, in_features, seed, dtype, bias)
        self.weight = torch.nn.Parameter(w[:, r * k:(r + 1) * k].contiguous().to(device))
        self.bias = torch.nn.Parameter(b.to(device)) if bias else None

    def forward(self, x):
        if not self.input_is_parallel:
            x = scatter_to_tensor_parallel_region(x, self.comm)
        if _fused_ok(x.reshape(-1, x.shape[-1]), self.weight, self.comm):
            # the TP all-reduce rides in the GEMM epilogue (tile-granular overlap)
            return _RowParallelFused.apply(x, self.weight, self.bias, self.comm)
        y = reduce_from_tensor_parallel_region(_LinearFn.apply(x, self.weight, None, self.comm), self.comm)
        return y + self.bias if self.bias is not None else y


class _GateUpSwiGLU(torch.autograd.Function):
    """``a = swiglu_pairs(x W^T)`` for a gate|up weight whose rows are interleaved (gate j,
    up j) pairs.  Forward: one GEMM whose epilogue also writes the gate (LDS-ring kernel,
    EPI 2), else GEMM + ``swiglu_pairs``; saves x, W and the GEMM output h.  Backward:
    ``swiglu_pairs_backward`` (one kernel) then dX / dW as ``_LinearFn``."""

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
        dh = swiglu_pairs_backward(h, da.reshape(-1, da.shape[-1]))
        if ctx.mfma:
            dx, dw = _linear_backward(dh, x2, w, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.comm)
        else:
            dx = dh @ w if ctx.needs_input_grad[0] else None
            dw = dh.t() @ x2 if ctx.needs_input_grad[1] else None
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

    def __init__(self, d_model: int, ffn: int, comm, device=None, dtype=torch.bfloat16, seed: int = 0):
        super().__init__()
        p, r = _size_rank(comm)
        if ffn % p:
            raise ValueError(f"ffn {ffn} not divisible by TP size {p}")
        k = ffn // p
        self.comm, self.p, self.r, self.ffn = comm, p, r, ffn
        self.gate_up = ColumnParallelLinear(d_model, 2 * ffn, comm, bias=False, device=device, dtype=dtype, seed=seed)
        full, _ = _init_full(2 * ffn, d_model, seed, dtype, False)
        with torch.no_grad():  # shard rows: gate r k + j at 2 j, up r k + j at 2 j + 1
            shard = torch.stack([full[r * k:(r + 1) * k], full[ffn + r * k:ffn + (r + 1) * k]], dim=1)
            self.gate_up.weight.copy_(shard.reshape(2 * k, d_model))
        self.down = RowParallelLinear(ffn, d_model, comm, bias=False, device=device, dtype=dtype, seed=seed + 1)

    def _fused_ok(self, x) -> bool:
        w = self.gate_up.weight
        return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
                and (w.shape[0] // 2) % 4 == 0)

    def forward(self, x):
        if self._fused_ok(x):
            a = _GateUpSwiGLU.apply(copy_to_tensor_parallel_region(x, self.comm), self.gate_up.weight, self.comm)
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


__all__ = ["ColumnParallelLinear", "RowParallelLinear", "ParallelSwiGLUMLP", "all_reduce_", "copy_to_tensor_parallel_region",
           "reduce_from_tensor_parallel_region", "gather_from_tensor_parallel_region",
           "scatter_to_tensor_parallel_region", "full_weight", "sharded_grad_full"]
