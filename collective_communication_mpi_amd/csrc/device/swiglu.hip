// Fused SwiGLU gate for the Llama-style MLP between the column-parallel gate|up GEMM
// and the row-parallel down GEMM (parallel/tensor_parallel.py ParallelSwiGLUMLP).
//
//   forward : a[t, j]  = silu(g) * u,            g = h[t, j], u = h[t, k + j]
//   backward: dh[t, j] = da * u * s * (1 + g (1 - s)),  dh[t, k + j] = da * silu(g)
//
// h is the [T, 2k] bf16 output of the gate|up GEMM (this rank's gate features in the
// first k columns, the matching up features in the next k).  Eager PyTorch spends
// ~10 passes on this (strided silu, mul, and in backward two mul, silu_backward, two
// zero-filled slice gradients and their sum: ~13 % of the TP MLP's GPU time,
// profiles/r3_gemm/tp_mlp_own_kernel_stats.md); here it is one read of h (+ da) and
// one write, 16-B vectors, fp32 math, one bf16 rounding per output.
//
// Grid: x = row t (no integer division), y = 256-vector column chunks.
//
// Interleaved layout (ParallelSwiGLUMLP): h[t, 2j] = gate j, h[t, 2j + 1] = up j, so
// the gate|up GEMM's own epilogue can apply the gate (gemm_w4.hip EPI 2,
// `gemm_nt_swiglu`): each 16-B row vector of C holds 4 whole pairs.  `*_il` kernels are
// the unfused forms of that layout (other GEMM routes) and its backward.
#include <pybind11/pybind11.h>

#include <cstdlib>

#include "common.hpp"
#include "gemm_common.hpp"
#include "ops.hpp"

namespace ccmpi {
namespace dev {

namespace {

__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));  // exp -> inf gives 0, exp -> 0 gives 1
}

__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  return pk_bf16(lo, hi);
}

__global__ void __launch_bounds__(256) k_swiglu_fwd(const uint16_t* __restrict__ h, uint16_t* __restrict__ a,
                                                    int kv, int64_t ldh, int64_t lda) {
  const int j = blockIdx.y * 256 + threadIdx.x;  // 8-element vector index within the row
  if (j >= kv) return;
  const int64_t t = blockIdx.x;
  const uint16_t* hr = h + t * ldh;
  const u32x4 g = *reinterpret_cast<const u32x4*>(hr + 8 * (int64_t)j);
  const u32x4 u = *reinterpret_cast<const u32x4*>(hr + 8 * ((int64_t)kv + j));
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float g0 = bf16_lo(g[i]), g1 = bf16_hi(g[i]);
    r[i] = pack_bf16(g0 * sigmoid_fast(g0) * bf16_lo(u[i]), g1 * sigmoid_fast(g1) * bf16_hi(u[i]));
  }
  *reinterpret_cast<u32x4*>(a + t * lda + 8 * (int64_t)j) = r;
}

__global__ void __launch_bounds__(256) k_swiglu_bwd(const uint16_t* __restrict__ h, const uint16_t* __restrict__ da,
                                                    uint16_t* __restrict__ dh, int kv, int64_t ldh, int64_t ldda,
                                                    int64_t lddh) {
  const int j = blockIdx.y * 256 + threadIdx.x;
  if (j >= kv) return;
  const int64_t t = blockIdx.x;
  const uint16_t* hr = h + t * ldh;
  const u32x4 g = *reinterpret_cast<const u32x4*>(hr + 8 * (int64_t)j);
  const u32x4 u = *reinterpret_cast<const u32x4*>(hr + 8 * ((int64_t)kv + j));
  const u32x4 d = *reinterpret_cast<const u32x4*>(da + t * ldda + 8 * (int64_t)j);
  u32x4 rg, ru;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float dg2[2], du2[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const float gv = half ? bf16_hi(g[i]) : bf16_lo(g[i]);
      const float uv = half ? bf16_hi(u[i]) : bf16_lo(u[i]);
      const float dv = half ? bf16_hi(d[i]) : bf16_lo(d[i]);
      const float s = sigmoid_fast(gv);
      du2[half] = dv * gv * s;
      dg2[half] = dv * uv * s * (1.0f + gv * (1.0f - s));
    }
    rg[i] = pack_bf16(dg2[0], dg2[1]);
    ru[i] = pack_bf16(du2[0], du2[1]);
  }
  uint16_t* dr = dh + t * lddh;
  *reinterpret_cast<u32x4*>(dr + 8 * (int64_t)j) = rg;
  *reinterpret_cast<u32x4*>(dr + 8 * ((int64_t)kv + j)) = ru;
}

// interleaved pairs: thread = 4 pairs (16 B of h, 8 B of a / da)
__global__ void __launch_bounds__(256) k_swiglu_fwd_il(const uint16_t* __restrict__ h, uint16_t* __restrict__ a,
                                                       int nv, int64_t ldh, int64_t lda) {
  const int j = blockIdx.y * 256 + threadIdx.x;
  if (j >= nv) return;
  const int64_t t = blockIdx.x;
  const u32x4 w = *reinterpret_cast<const u32x4*>(h + t * ldh + 8 * (int64_t)j);
  float r[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float gv = bf16_lo(w[q]);
    r[q] = gv * sigmoid_fast(gv) * bf16_hi(w[q]);
  }
  *reinterpret_cast<uint2*>(a + t * lda + 4 * (int64_t)j) = uint2{pack_bf16(r[0], r[1]), pack_bf16(r[2], r[3])};
}

__global__ void __launch_bounds__(256) k_swiglu_bwd_il(const uint16_t* __restrict__ h, const uint16_t* __restrict__ da,
                                                       uint16_t* __restrict__ dh, int nv, int64_t ldh, int64_t ldda,
                                                       int64_t lddh) {
  const int j = blockIdx.y * 256 + threadIdx.x;
  if (j >= nv) return;
  const int64_t t = blockIdx.x;
  const u32x4 w = *reinterpret_cast<const u32x4*>(h + t * ldh + 8 * (int64_t)j);
  const uint2 d2 = *reinterpret_cast<const uint2*>(da + t * ldda + 4 * (int64_t)j);
  const uint32_t dd[2] = {d2.x, d2.y};
  u32x4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float gv = bf16_lo(w[q]), uv = bf16_hi(w[q]);
    const float dv = (q & 1) ? bf16_hi(dd[q >> 1]) : bf16_lo(dd[q >> 1]);
    const float sg = sigmoid_fast(gv);
    r[q] = pack_bf16(dv * uv * sg * (1.0f + gv * (1.0f - sg)), dv * gv * sg);
  }
  *reinterpret_cast<u32x4*>(dh + t * lddh + 8 * (int64_t)j) = r;
}

// The same, plus dh^T [2k, T] for the weight-gradient GEMM dW = dh^T X (which then runs
// on the N-layout pair ring instead of the K-major one, with no separate transpose pass):
// a 64-row x 64-column tile of dh per workgroup, written row-major straight away and
// through an LDS tile (33-word row stride: conflict-free column gathers) transposed,
// 16-B stores both ways.  T % 8 == 0.
template <int R>  // rows per tile (a multiple of 32)
__global__ void __launch_bounds__(256) k_swiglu_bwd_il_t(const uint16_t* __restrict__ h, const uint16_t* __restrict__ da,
                                                         uint16_t* __restrict__ dh, uint16_t* __restrict__ dht, int T,
                                                         int n, int64_t ldh, int64_t ldda, int64_t lddh, int64_t ldt) {
  constexpr int S = 66;  // LDS row stride, elements
  __shared__ uint32_t tile[R * S / 2];
  const int t = threadIdx.x;
  const int r0 = blockIdx.y * R, c0 = blockIdx.x * 64;
  const int lr = t >> 3, lc = (t & 7) * 8;
#pragma unroll
  for (int hh = 0; hh < R / 32; ++hh) {
    const int row = lr + 32 * hh;
    u32x4 r = u32x4{0u, 0u, 0u, 0u};
    if (r0 + row < T && c0 + lc < n) {
      const int64_t tr = r0 + row;
      const u32x4 w = *reinterpret_cast<const u32x4*>(h + tr * ldh + c0 + lc);
      const uint2 d2 = *reinterpret_cast<const uint2*>(da + tr * ldda + (c0 + lc) / 2);
      const uint32_t dd[2] = {d2.x, d2.y};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gv = bf16_lo(w[q]), uv = bf16_hi(w[q]);
        const float dv = (q & 1) ? bf16_hi(dd[q >> 1]) : bf16_lo(dd[q >> 1]);
        const float sg = sigmoid_fast(gv);
        r[q] = pack_bf16(dv * uv * sg * (1.0f + gv * (1.0f - sg)), dv * gv * sg);
      }
      *reinterpret_cast<u32x4*>(dh + tr * lddh + c0 + lc) = r;
    }
    uint32_t* d = tile + (row * S + lc) / 2;
    d[0] = r[0]; d[1] = r[1]; d[2] = r[2]; d[3] = r[3];
  }
  __syncthreads();
  const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
  // dh^T row c0 + oc, columns r0 + 8 q ..: R / 8 lanes per destination row
  constexpr int QL = R / 8, RPW = 256 / QL;
#pragma unroll
  for (int hh = 0; hh < 64 / RPW; ++hh) {
    const int oc = t / QL + RPW * hh, q = t % QL;
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
      o[m] = (uint32_t)t16[(8 * q + 2 * m) * S + oc] | ((uint32_t)t16[(8 * q + 2 * m + 1) * S + oc] << 16);
    if (c0 + oc < n && r0 + 8 * q < T)
      *reinterpret_cast<uint4*>(dht + (int64_t)(c0 + oc) * ldt + r0 + 8 * q) = uint4{o[0], o[1], o[2], o[3]};
  }
}

void check(uint64_t T, uint64_t k, uint64_t ptrs, uint64_t lds) {
  if (k % 8 || (ptrs | (lds * 2)) % 16)
    throw std::invalid_argument("swiglu: k % 8 == 0, 16-B aligned pointers and row strides required");
  if (T > 0x7fffffffull || k / 8 > 256ull * 65535ull)
    throw std::invalid_argument("swiglu: too many rows or columns for the grid");
}

void check_il(uint64_t T, uint64_t k, uint64_t hptrs, uint64_t hld, uint64_t aptrs, uint64_t ald) {
  if (k % 4 || (hptrs | (hld * 2)) % 16 || (aptrs | (ald * 2)) % 8)
    throw std::invalid_argument("swiglu (interleaved): k % 4 == 0, 16-B aligned h rows, 8-B aligned a rows required");
  if (T > 0x7fffffffull || k / 4 > 256ull * 65535ull)
    throw std::invalid_argument("swiglu: too many rows or columns for the grid");
}

}  // namespace

void register_swiglu_ops(pybind11::module_& m) {
  m.def("swiglu_fwd_il", [](uint64_t h, uint64_t a, uint64_t T, uint64_t k, int64_t ldh, int64_t lda, uint64_t stream) {
    check_il(T, k, h, (uint64_t)ldh, a, (uint64_t)lda);
    if (T == 0 || k == 0) return;
    const int nv = (int)(k / 4);
    hipLaunchKernelGGL(k_swiglu_fwd_il, dim3((unsigned)T, (nv + 255) / 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint16_t*>(h),
                       reinterpret_cast<uint16_t*>(a), nv, ldh, lda);
    CCMPI_HIP_CHECK(hipGetLastError());
  }, "a[T, k] = silu(h[:, 0::2]) * h[:, 1::2] (interleaved gate/up pairs, bf16)");
  m.def("swiglu_bwd_il", [](uint64_t h, uint64_t da, uint64_t dh, uint64_t T, uint64_t k, int64_t ldh, int64_t ldda,
                            int64_t lddh, uint64_t stream) {
    check_il(T, k, h | dh, (uint64_t)(ldh | lddh), da, (uint64_t)ldda);
    if (T == 0 || k == 0) return;
    const int nv = (int)(k / 4);
    hipLaunchKernelGGL(k_swiglu_bwd_il, dim3((unsigned)T, (nv + 255) / 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint16_t*>(h),
                       reinterpret_cast<const uint16_t*>(da), reinterpret_cast<uint16_t*>(dh), nv, ldh, ldda, lddh);
    CCMPI_HIP_CHECK(hipGetLastError());
  }, "dh[T, 2k] (interleaved pairs) from h[T, 2k] and da[T, k]");
  m.def("swiglu_bwd_il_t", [](uint64_t h, uint64_t da, uint64_t dh, uint64_t dht, uint64_t T, uint64_t k, int64_t ldh,
                              int64_t ldda, int64_t lddh, int64_t ldt, uint64_t stream) {
    check_il(T, k, h | dh | dht, (uint64_t)(ldh | lddh | ldt), da, (uint64_t)ldda);
    if (T % 8) throw std::invalid_argument("swiglu_bwd_il_t: T % 8 == 0 required");
    if (T == 0 || k == 0) return;
    const int n = (int)(2 * k);
    // 64-row tiles: 128-row ones measured 3 % slower (profiles/r4_swiglu_t)
    constexpr int R = 64;
    hipLaunchKernelGGL(k_swiglu_bwd_il_t<R>, dim3((n + 63) / 64, (unsigned)((T + R - 1) / R)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint16_t*>(h),
                       reinterpret_cast<const uint16_t*>(da), reinterpret_cast<uint16_t*>(dh),
                       reinterpret_cast<uint16_t*>(dht), (int)T, n, ldh, ldda, lddh, ldt);
    CCMPI_HIP_CHECK(hipGetLastError());
  }, "swiglu_bwd_il plus dh^T [2k, T] (the dW GEMM's N-layout operand)");
  // C[M, N] = A[M, K] B[N, K]^T (bf16) on the LDS-ring kernel with the SwiGLU epilogue:
  // glu[M, N / 2] from C's interleaved (gate, up) column pairs.  False (nothing launched)
  // when the ring kernel's fast form does not apply; the caller then runs gemm_nt +
  // swiglu_fwd_il.
  m.def("gemm_nt_swiglu", [](uint64_t A, uint64_t B, uint64_t C, uint64_t glu, int M, int N, int K, int lda, int ldb,
                             int ldc, int ldglu, uint64_t stream) {
    if (M <= 0 || N <= 0) return true;
    gemm::GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B),
                     reinterpret_cast<void*>(C), nullptr, M, N, K, lda, ldb, ldc, 1.0f, 0, 0, 0, 1, 1};
    if (N % 8 || glu % 8 || ldglu % 4 || (int64_t)ldglu * 2 < N / 2 * 2 || !gemm::gemm_ring_ok(g, 0, 0) ||
        !gemm::gemm_w4_ok(g) || !gemm::gemm_w4r_fast(g))
      return false;
    gemm::launch_gemm_ring(g, 0, 0, reinterpret_cast<hipStream_t>(stream), reinterpret_cast<uint16_t*>(glu), ldglu);
    CCMPI_HIP_CHECK(hipGetLastError());
    return true;
  }, "bf16 NT GEMM with the SwiGLU gate of interleaved column pairs in its epilogue (ring kernel)");
  m.def("swiglu_fwd", [](uint64_t h, uint64_t a, uint64_t T, uint64_t k, int64_t ldh, int64_t lda, uint64_t stream) {
    check(T, k, h | a, (uint64_t)(ldh | lda));
    if (T == 0 || k == 0) return;
    const int kv = (int)(k / 8);
    hipLaunchKernelGGL(k_swiglu_fwd, dim3((unsigned)T, (kv + 255) / 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint16_t*>(h),
                       reinterpret_cast<uint16_t*>(a), kv, ldh, lda);
    CCMPI_HIP_CHECK(hipGetLastError());
  }, "a[T, k] = silu(h[:, :k]) * h[:, k:2k] (bf16, element strides ldh / lda)");
  m.def("swiglu_bwd", [](uint64_t h, uint64_t da, uint64_t dh, uint64_t T, uint64_t k, int64_t ldh, int64_t ldda,
                         int64_t lddh, uint64_t stream) {
    check(T, k, h | da | dh, (uint64_t)(ldh | ldda | lddh));
    if (T == 0 || k == 0) return;
    const int kv = (int)(k / 8);
    hipLaunchKernelGGL(k_swiglu_bwd, dim3((unsigned)T, (kv + 255) / 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint16_t*>(h),
                       reinterpret_cast<const uint16_t*>(da), reinterpret_cast<uint16_t*>(dh), kv, ldh, ldda, lddh);
    CCMPI_HIP_CHECK(hipGetLastError());
  }, "dh[T, 2k] from h[T, 2k] and da[T, k] (SwiGLU backward, bf16)");
}

}  // namespace dev
}  // namespace ccmpi
