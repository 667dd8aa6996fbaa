"""Python entry points of the device kernels (csrc/device/*.hip)."""
from __future__ import annotations

import os
from typing import Optional

import torch

from .. import _native

_ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2}


def _D():
    return _native.device()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


_TN_VARIANT = None  # tests / benchmarks: force the TN kernel (0 = 128x128, 1 = 256x256 ping-pong)


def set_tn_variant(v):
    global _TN_VARIANT
    _TN_VARIANT = v


def _auto_splitk(tiles: int, K: int) -> int:
    """Split K until the grid has ~2 workgroups per CU, keeping >= 4 K-tiles per split."""
    nk = (K + 63) // 64
    want = max(1, 512 // max(tiles, 1))
    return int(max(1, min(want, nk // 4, 32)))


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
            alpha: float = 1.0, accumulate: bool = False, act: Optional[str] = None,
            out_dtype: torch.dtype = torch.bfloat16, splitk: Optional[int] = None) -> torch.Tensor:
    """``out = act(alpha * a @ b.T + bias) (+ out)`` on MFMA (v_mfma_f32_16x16x32_bf16).

    a: [M, K] bf16 row-major (row stride may exceed K), b: [N, K] bf16; K % 8 == 0.
    bias: [N] fp32 or bf16.  out: [M, N] bf16 or fp32 (fp32 accumulate inside).
    """
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm_nt expects bf16 operands")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"gemm_nt shape mismatch: {tuple(a.shape)} x {tuple(b.shape)}^T")
    if a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("gemm_nt operands must be K-contiguous")
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs an output tensor")
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    if out.stride(1) != 1 or out.shape != (M, N):
        raise ValueError("gemm_nt output must be [M, N] with unit column stride")
    if out.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("gemm_nt output must be bf16 or fp32")
    bias_kind = 0
    bias_ptr = 0
    if bias is not None:
        bias_kind = 1 if bias.dtype == torch.float32 else 2
        if bias.dtype not in (torch.float32, torch.bfloat16) or not bias.is_contiguous() or bias.numel() != N:
            raise ValueError("bias must be a contiguous [N] fp32/bf16 tensor")
        bias_ptr = bias.data_ptr()
    if splitk is None:
        fp32_plain = out.dtype == torch.float32 and act is None
        splitk = _auto_splitk(((M + 127) // 128) * ((N + 127) // 128), K) if fp32_plain else 1
    _D().gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), bias_ptr, M, N, K, a.stride(0), b.stride(0),
                 out.stride(0), float(alpha), bool(accumulate), bias_kind, _ACT[act], out.dtype == torch.bfloat16,
                 int(splitk), _stream(a))
    return out


def gemm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, alpha: float = 1.0,
            accumulate: bool = False, splitk: Optional[int] = None, tail: Optional[torch.Tensor] = None,
            workspace: Optional[bool] = None) -> torch.Tensor:
    """``out[N1, N2] (+)= alpha * a[M, N1].T @ b[M, N2]`` (weight gradients dW = dY^T X) in fp32,
    reading both operands M-major through ds_read_b64_tr_b16 (no transposes).

    ``tail``: split the result by columns -- ``out`` (``[N1, c]``, accumulated if
    ``accumulate``) receives columns ``< c`` and ``tail`` (``[N1, N2 - c]``,
    overwritten) the rest, straight from the split-K reduction (one GEMM over a
    row-concatenated operand ``b = [X | Y]`` gives ``a^T X`` and ``a^T Y``).

    ``workspace``: split-K partials through a workspace + one reduction pass (True)
    or fp32 atomics into ``out`` (False); default by output size."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm_tn expects bf16 operands")
    if a.dim() != 2 or b.dim() != 2 or a.shape[0] != b.shape[0] or a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError(f"gemm_tn shape mismatch: {tuple(a.shape)}^T x {tuple(b.shape)}")
    M, N1 = a.shape
    N2 = b.shape[1]
    csplit = 0
    if tail is not None:
        if out is None:
            raise ValueError("gemm_tn: tail needs an explicit out")
        csplit = out.shape[1]
        if (tail.dtype != torch.float32 or tail.shape != (N1, N2 - csplit) or tail.stride(1) != 1
                or csplit % 4 or tail.stride(0) % 4 or tail.data_ptr() % 16):
            raise ValueError("gemm_tn tail must be fp32 [N1, N2 - out cols], 16-B aligned rows, out cols % 4 == 0")
        if out.dtype != torch.float32 or out.shape[0] != N1 or out.stride(1) != 1:
            raise ValueError("gemm_tn output must be fp32 [N1, c] with unit column stride")
    elif out is None:
        if accumulate:
            raise ValueError("accumulate needs an output tensor")
        out = torch.empty((N1, N2), dtype=torch.float32, device=a.device)
    if tail is None and (out.dtype != torch.float32 or out.shape != (N1, N2) or out.stride(1) != 1):
        raise ValueError("gemm_tn output must be fp32 [N1, N2] with unit column stride")
    # variant 1 (256x256 ping-pong TN) is opt-in: measured slower than the 128x128 TN kernel on
    # every shape tried (benchmarks/gemm_tn_splitk.py, profiles/r1_gemm_fastepi/tn_variants.txt)
    variant = _TN_VARIANT if _TN_VARIANT is not None else 0
    if variant == 1 and not (M % 128 == 0 and N1 >= 256 and N2 >= 256):
        variant = 0
    if splitk is None:
        if variant == 1:  # 256x256 tiles: split K until ~1 workgroup per CU, >= 2 K-tile pairs per split
            tiles = ((N1 + 255) // 256) * ((N2 + 255) // 256)
            splitk = int(max(1, min(256 // max(tiles, 1), M // 256, 64)))
        else:
            splitk = _auto_splitk(((N1 + 127) // 128) * ((N2 + 127) // 128), M)
    if tail is not None:
        splitk = max(2, splitk)  # the column split happens in the split-K reduction
    ws = 0
    # large outputs: partials in a workspace + one reduction pass instead of fp32 atomics
    # (dW_qkv 768x768: 80 -> 68 us); small outputs keep the atomics (one launch fewer)
    use_ws = workspace if workspace is not None else (variant == 1 or N1 * N2 >= (1 << 18) or tail is not None)
    if splitk > 1 and N2 % 4 == 0 and (use_ws or tail is not None):
        ws = torch.empty(splitk * N1 * N2, dtype=torch.float32, device=a.device).data_ptr()
    _D().gemm_tn(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N1, N2, a.stride(0), b.stride(0), out.stride(0),
                 float(alpha), bool(accumulate), int(splitk), _stream(a), ws, int(variant),
                 0 if tail is None else tail.data_ptr(), 0 if tail is None else tail.stride(0), csplit)
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x[..., K] @ w[N, K].T + bias`` with the MFMA GEMM (bf16 out)."""
    lead = x.shape[:-1]
    y = gemm_nt(x.reshape(-1, x.shape[-1]), w, out=None if out is None else out.reshape(-1, w.shape[0]),
                bias=bias, act=act)
    return y.reshape(*lead, w.shape[0])


def gemm_ring(a: torch.Tensor, b: torch.Tensor, ta: bool, tb: bool, out: Optional[torch.Tensor] = None,
              alpha: float = 1.0, accumulate: bool = False, out_dtype: torch.dtype = torch.bfloat16,
              a_nt: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """``out = alpha * op(a) @ op(b).T (+ out)`` on the four-wave LDS-ring MFMA kernel
    (csrc/device/gemm_w4.hip), with either operand K-major: op(a) = a.T if ``ta`` (a is
    [K, M]) else a ([M, K]); op(b) = b.T if ``tb`` (b is [K, N]) else b ([N, K]).
    dX = dY W is ``gemm_ring(dY, W, False, True)``, dW = dY^T X is
    ``gemm_ring(dY, X, True, True)``: no transposes.  Returns None when the kernel does
    not apply (K % 64, 16-B alignment, > 2 GiB operands): the caller falls back.
    ``a_nt``: op(a) already in N layout (``a.T`` contiguous, e.g. the dh^T the SwiGLU
    backward writes): the N-layout pair ring runs on it, no transpose of ``a``."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2:
        raise TypeError("gemm_ring expects 2-D bf16 operands")
    if a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("gemm_ring operands must have unit inner stride")
    M, K = (a.shape[1], a.shape[0]) if ta else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[1], b.shape[0]) if tb else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm_ring shape mismatch: op(a) {M}x{K}, op(b) {N}x{Kb}")
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs an output tensor")
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    if out.shape != (M, N) or out.stride(1) != 1 or out.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("gemm_ring output must be [M, N] bf16/fp32 with unit column stride")
    route = os.environ.get("CCMPI_KMAJOR_ROUTE", "pair")
    if ta and route == "pair":
        # dW = dY^T X with both operands M-major on the pair-slot ring's TA (+ TB) form: no
        # transposes at all (an N-layout copy the producer wrote is not needed either).
        # Llama-3-8B MLP at T = 4096: dW_down 0.369 ms against 0.464 ms for both operands
        # transposed, the whole block forward + backward 3.334 ms against 3.395 ms
        # (profiles/r5_fourth).  CCMPI_KMAJOR_ROUTE=transpose: the round-4 route
        ok = _D().gemm_ring(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                            out.stride(0), 1, int(tb), float(alpha), bool(accumulate), out.dtype == torch.bfloat16,
                            _stream(a))
        if ok:
            return out
    if ta and (a_nt is not None or _kmajor_via_transpose(M, N, K, a, b)):
        # K-major A transposed first (k_transpose16_v, ~6 TB/s) -- or taken from a_nt, the
        # N-layout copy its producer wrote -- then the pair-slot ring: its whole-line DMA
        # pieces and one ds_read_b128 per fragment beat the 4-slot K-major ring's two
        # transposed LDS reads per fragment (profiles/r4_bwd).  A K-major B stays K-major:
        # the pair ring reads it directly (its dX = dY W form), so dW = dY^T X transposes
        # at most dY (CCMPI_WGRAD_B=transpose: the old route, both operands transposed)
        at = a_nt if a_nt is not None else transpose(a)
        if tb and os.environ.get("CCMPI_WGRAD_B", "kmajor") == "kmajor":
            return gemm_ring(at, b, False, True, out=out, alpha=alpha, accumulate=accumulate, out_dtype=out_dtype)
        bt = transpose(b) if tb else b
        return gemm_ring(at, bt, False, False, out=out, alpha=alpha, accumulate=accumulate, out_dtype=out_dtype)
    ok = _D().gemm_ring(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0), out.stride(0),
                        int(ta), int(tb), float(alpha), bool(accumulate), out.dtype == torch.bfloat16, _stream(a))
    return out if ok else None


def _kmajor_via_transpose(M: int, N: int, K: int, a: torch.Tensor, b: torch.Tensor) -> bool:
    """Route a K-major ring GEMM through transposed copies (CCMPI_KMAJOR_ROUTE=transpose,
    read per call; default ``pair``: the pair ring reads K-major operands itself; ``ring``: the
    4-slot K-major kernel): K-major A (the dW = dY^T X form), large GEMMs only, and not long
    K.  dX = dY W (K-major B only) stays on the ring: a transposed weight copy + the pair ring
    measured no faster (profiles/r4_bwd)."""
    if os.environ.get("CCMPI_KMAJOR_ROUTE", "pair") != "transpose":
        return False
    dmin = int(os.environ.get("CCMPI_KMAJOR_MIN_DIM", 1024))  # (tests lower both thresholds)
    return (M >= dmin and N >= dmin and K <= 16384 and K % 8 == 0 and M % 8 == 0 and N % 8 == 0
            and M * N * K >= int(os.environ.get("CCMPI_KMAJOR_MIN_MACS", 1 << 33))
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0)


def transpose(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """2-D transpose of a 16-bit tensor: 16-B register-transpose kernel when the shape and
    strides are multiples of 8 elements (k_transpose16_v), else the LDS-tiled one."""
    if x.dim() != 2 or x.element_size() != 2 or x.stride(1) != 1:
        raise ValueError("transpose expects a 2-D row-contiguous 16-bit tensor")
    R, C = x.shape
    if out is None:
        out = torch.empty((C, R), dtype=x.dtype, device=x.device)
    _D().transpose16(x.data_ptr(), out.data_ptr(), R, C, x.stride(0), out.stride(0), _stream(x))
    return out


def _swiglu_rows(t: torch.Tensor) -> torch.Tensor:
    """2-D view ``[rows, cols]`` with unit column stride (copies only if it must)."""
    t2 = t.reshape(-1, t.shape[-1])
    ok = t2.stride(1) == 1 and t2.stride(0) % 8 == 0 and t2.data_ptr() % 16 == 0
    return t2 if ok else t2.contiguous()


class _SwiGLU(torch.autograd.Function):
    """``silu(h[..., :k]) * h[..., k:]`` in one HIP kernel each way (csrc/device/swiglu.hip);
    saves only ``h`` (the gate|up GEMM output), backward writes ``dh`` in one pass."""

    @staticmethod
    def forward(ctx, h):
        h2 = _swiglu_rows(h)
        k = h2.shape[1] // 2
        a = torch.empty(*h.shape[:-1], k, dtype=h.dtype, device=h.device)
        _D().swiglu_fwd(h2.data_ptr(), a.data_ptr(), h2.shape[0], k, h2.stride(0), k, _stream(h2))
        ctx.save_for_backward(h2)
        ctx.lead = h.shape[:-1]
        return a

    @staticmethod
    def backward(ctx, da):
        (h2,) = ctx.saved_tensors
        k = h2.shape[1] // 2
        da2 = _swiglu_rows(da)
        dh = torch.empty(*ctx.lead, 2 * k, dtype=h2.dtype, device=h2.device)
        _D().swiglu_bwd(h2.data_ptr(), da2.data_ptr(), dh.data_ptr(), h2.shape[0], k, h2.stride(0), da2.stride(0),
                        2 * k, _stream(h2))
        return dh


def swiglu(h: torch.Tensor) -> torch.Tensor:
    """SwiGLU gate of a ``[..., 2k]`` gate|up tensor: ``silu(h[..., :k]) * h[..., k:]``.

    CUDA bf16 with ``k % 8 == 0`` runs the fused HIP kernels (fp32 math, one bf16
    rounding); anything else (CPU, other dtypes) is computed by torch ops."""
    if h.shape[-1] % 2:
        raise ValueError("swiglu needs an even last dimension (gate | up)")
    k = h.shape[-1] // 2
    if h.is_cuda and h.dtype == torch.bfloat16 and k % 8 == 0 and h.data_ptr() % 16 == 0:
        return _SwiGLU.apply(h)
    return torch.nn.functional.silu(h[..., :k]) * h[..., k:]


def swiglu_pairs(h: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """SwiGLU gate of interleaved (gate, up) pairs: ``silu(h[:, 0::2]) * h[:, 1::2]``
    (``h`` [T, 2k] bf16 CUDA, row-contiguous; one HIP kernel, no autograd)."""
    T, n = h.shape
    if out is None:
        out = torch.empty((T, n // 2), dtype=h.dtype, device=h.device)
    _D().swiglu_fwd_il(h.data_ptr(), out.data_ptr(), T, n // 2, h.stride(0), out.stride(0), _stream(h))
    return out


def swiglu_pairs_backward(h: torch.Tensor, da: torch.Tensor, transposed: bool = False):
    """Gradient of ``swiglu_pairs`` w.r.t. its interleaved input (one HIP kernel).  With
    ``transposed`` (T % 8 == 0): returns ``(dh, dh^T)``, the transposed copy written by the
    same kernel (the weight-gradient GEMM's N-layout operand, no separate transpose)."""
    T, n = h.shape
    da = da if (da.stride(1) == 1 and da.stride(0) % 4 == 0) else da.contiguous()
    dh = torch.empty_like(h)
    if transposed:
        dht = torch.empty(n, T, device=h.device, dtype=h.dtype)
        _D().swiglu_bwd_il_t(h.data_ptr(), da.data_ptr(), dh.data_ptr(), dht.data_ptr(), T, n // 2, h.stride(0),
                             da.stride(0), dh.stride(0), dht.stride(0), _stream(h))
        return dh, dht
    _D().swiglu_bwd_il(h.data_ptr(), da.data_ptr(), dh.data_ptr(), T, n // 2, h.stride(0), da.stride(0),
                       dh.stride(0), _stream(h))
    return dh


def gemm_nt_swiglu(a: torch.Tensor, b: torch.Tensor, h: torch.Tensor, glu: torch.Tensor) -> bool:
    """``h = a @ b.T`` (bf16) with the SwiGLU gate of h's interleaved column pairs written
    to ``glu`` by the GEMM's own epilogue (LDS-ring kernel, csrc/device/gemm_w4.hip EPI 2).
    Returns False (nothing launched) when the ring kernel's fast form does not apply."""
    M, K = a.shape
    N = b.shape[0]
    if not (a.stride(1) == 1 and b.stride(1) == 1 and h.shape == (M, N) and h.stride(1) == 1
            and glu.shape == (M, N // 2) and glu.stride(1) == 1):
        return False
    return bool(_D().gemm_nt_swiglu(a.data_ptr(), b.data_ptr(), h.data_ptr(), glu.data_ptr(), M, N, K, a.stride(0),
                                    b.stride(0), h.stride(0), glu.stride(0), _stream(a)))


def interleave_lastaxis(stage: torch.Tensor, p: int) -> torch.Tensor:
    """``[p, *lead, k] -> [*lead, p*k]`` (np.concatenate(parts, axis=-1))."""
    stage = stage.contiguous()
    lead, k = stage.shape[1:-1], stage.shape[-1]
    M = stage[0].numel() // max(k, 1)
    out = torch.empty(*lead, p * k, dtype=stage.dtype, device=stage.device)
    _D().interleave_lastaxis(stage.data_ptr(), out.data_ptr(), M, p, k * stage.element_size(), _stream(stage))
    return out


def deinterleave_lastaxis(x: torch.Tensor, p: int) -> torch.Tensor:
    """``[*lead, p*k] -> [p, *lead, k]`` (np.stack(np.split(x, p, axis=-1)))."""
    x = x.contiguous()
    n = x.shape[-1]
    if n % p:
        raise ValueError("last axis not divisible by p")
    k = n // p
    M = x.numel() // max(n, 1)
    out = torch.empty(p, *x.shape[:-1], k, dtype=x.dtype, device=x.device)
    _D().deinterleave_lastaxis(x.data_ptr(), out.data_ptr(), M, p, k * x.element_size(), _stream(x))
    return out
