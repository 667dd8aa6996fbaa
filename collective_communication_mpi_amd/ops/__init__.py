"""Device ops backed by the hand-written HIP kernels of ``_device`` (gfx950).

Every op fails loudly (raises) when the extension is missing or an input
violates a kernel precondition; there is no silent eager fallback."""
from .kernels import (  # noqa: F401
    gemm_nt,
    gemm_tn,
    gemm_ring,
    linear,
    swiglu,
    swiglu_pairs,
    swiglu_pairs_backward,
    gemm_nt_swiglu,
    transpose,
    interleave_lastaxis,
    deinterleave_lastaxis,
)
