// bf16 GEMM on CDNA4 matrix cores with fused epilogue, for the TP layers of
// the DP x TP harness (fc_q/k/v column-parallel, fc_o row-parallel, patch
// embedding).  The reference leaves this compute "taken care of" elsewhere
// (README.md:173-175); here it is the hot op of the training step.
//
//   C[M,N] = act(alpha * A[M,K] . B[N,K]^T + bias[N]) (+ C if accumulate)
//
// A and B are both K-contiguous ("NT"; PyTorch Linear weights are [out, in]),
// bf16, rows 16-B aligned (K % 8 == 0, lda/ldb % 8 == 0).  Backward passes
// feed transposed copies made by k_transpose (below).
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves as 2x2, each
// wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles), BK = 64, two LDS buffers
// (64 KiB).  Global -> register loads of tile k+1 are issued before the MFMAs
// of tile k and written to the other LDS buffer after them (one barrier per
// K-step).  LDS rows are 128 B; the 16-B chunk index is XOR-swizzled with
// (row & 7) so a 16-lane ds_read_b128 group touches 8 different slots.
// Workgroup ids are remapped so that consecutive N-tiles of one M-row of
// tiles land on the same XCD (shared A panel in that XCD's L2).
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "common.hpp"
#include "gemm_common.hpp"
#include "ops.hpp"

namespace ccmpi {
namespace dev {

namespace {
using namespace gemm;

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
bool g_use_glds = std::getenv("CCMPI_GEMM_NO_GLDS") == nullptr;  // A/B switch (benchmarks)
bool g_direct_epi = std::getenv("CCMPI_GEMM_STAGED_EPI") == nullptr;  // LDS-free epilogue (A/B switch)
// (round 1 also carried a BK = 32, a multi-stage (3-5 x 16 KiB) and a persistent
// form of the 128x128 kernel; all measured slower or no faster
// (profiles/r1_qkv_reassoc/qkv_shapes2.txt, profiles/r1_gemm_fastepi) and were removed)
// kernel choice for gemm_nt: 0 auto, 1 = 128x128 only, 2 = 256x256 / 3 = 256x128 / 4 = 256x192 whenever legal
int g_kernel = std::getenv("CCMPI_GEMM_KERNEL") ? std::atoi(std::getenv("CCMPI_GEMM_KERNEL")) : 0;
constexpr int kRowBytes = BK * 2;  // 128 B per LDS row

// Shared epilogue of the 128x128 kernels: lane holds D[4*(lane>>4) + r][lane & 15]
// of each 16x16 tile.  Stage the (alpha, bias, act)-applied fp32 tile through
// LDS (the A/B buffers are dead now), then write whole rows (store_rows).
__device__ __forceinline__ void store_tile(const GemmArgs& g, floatx4 (&acc)[4][4], unsigned char* smem, int bm,
                                           int bn, int wm, int wn, int split, int t, int lane) {
  float* tile = reinterpret_cast<float*>(smem);
  constexpr int TS = BN + 4;  // fp32 row stride in LDS
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wn + j * 16 + (lane & 15);
    const float b = load_bias(g, bn + cl, split);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(wm + i * 16 + (lane >> 4) * 4 + r) * TS + cl] = epi(g, acc[i][j][r], b);
  }
  __syncthreads();
  store_rows<BM, BN, NT>(g, tile, TS, bm, bn, t);
}

// Branch-free staged epilogue of the weight-gradient GEMM (fp32 C, alpha only):
// ATOMIC = split-K partial sums as lane-consecutive fp32 atomics, otherwise
// plain (or accumulating) 16-B row stores.
template <bool ATOMIC, bool ACCUM>
__device__ __forceinline__ void store_tile_f32(const GemmArgs& g, floatx4 (&acc)[4][4], unsigned char* smem, int bm,
                                              int bn, int wm, int wn, int t, int lane) {
  float* tile = reinterpret_cast<float*>(smem);
  constexpr int TS = BN + 4;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        tile[(wm + i * 16 + (lane >> 4) * 4 + r) * TS + wn + j * 16 + (lane & 15)] = g.alpha * acc[i][j][r];
  __syncthreads();
  if constexpr (ATOMIC) {
    for (int idx = t; idx < BM * BN; idx += NT) {
      const int rl = idx / BN, cl = idx % BN;
      const int row = bm + rl, col = bn + cl;
      if (row < g.M && col < g.N) atomicAdd(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col, tile[rl * TS + cl]);
    }
  } else {
    for (int idx = t; idx < BM * (BN / 4); idx += NT) {
      const int rl = idx / (BN / 4), cl = (idx % (BN / 4)) * 4;
      const int row = bm + rl, col = bn + cl;
      if (row >= g.M || col >= g.N) continue;
      float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col);
      float4 v = make_float4(tile[rl * TS + cl], tile[rl * TS + cl + 1], tile[rl * TS + cl + 2], tile[rl * TS + cl + 3]);
      if constexpr (ACCUM) {
        const float4 o = *C;
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      *C = v;
    }
  }
}

// Direct (LDS-free) epilogue for kernels that swap the MFMA operands and stage
// B rows in the "pair" permutation: LDS row 32p + 16h + q of the B tile holds
// output column 32p + 8*(q >> 2) + 4h + (q & 3).  The accumulator of tile
// (i, j = 2p + h) then holds C[row0 + 16i + (lane & 15)][col0 + 32p + 8*(lane >> 4) + 4h + r],
// i.e. 8 consecutive columns of one row per lane and pair: one 16-B vector store
// (bf16) or two (fp32).  Split-K partials go out as fp32 atomics.
__device__ __forceinline__ int pair_perm(int r) {
  return (r & ~31) | (((r & 15) >> 2) << 3) | (((r >> 4) & 1) << 2) | (r & 3);
}

__device__ __forceinline__ void store_direct(const GemmArgs& g, const floatx4 (&acc)[4][4], int row0, int col0, int split,
                                             int lane) {
  const int c = lane & 15, gq = lane >> 4;
  const int es = g.out_bf16 ? 2 : 4;
  const bool vec_ok = (((uint64_t)g.C | ((uint64_t)g.ldc * es)) % 16) == 0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int col = col0 + 32 * p + 8 * gq;
    if (col >= g.N) continue;
    float bias[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[e] = load_bias(g, col + e, split);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + 16 * i + c;
      if (row >= g.M) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = epi(g, acc[i][2 * p + (e >> 2)][e & 3], bias[e]);
      if (g.splitk > 1) {
        float* C = reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col;
        for (int e = 0; e < 8 && col + e < g.N; ++e) atomicAdd(C + e, v[e]);
      } else if (vec_ok && col + 8 <= g.N) {
        if (g.out_bf16) {
          uint16_t* C = reinterpret_cast<uint16_t*>(g.C) + (size_t)row * g.ldc + col;
          if (g.accumulate) {
            const uint4 o = *reinterpret_cast<const uint4*>(C);
            const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) { v[2 * q] += bf16_lo(ow[q]); v[2 * q + 1] += bf16_hi(ow[q]); }
          }
          uint32_t w[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) w[q] = pk_bf16(v[2 * q], v[2 * q + 1]);
          *reinterpret_cast<uint4*>(C) = uint4{w[0], w[1], w[2], w[3]};
        } else {
          float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col);
          float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
          if (g.accumulate) {
            const float4 p0 = C[0], p1 = C[1];
            o0.x += p0.x; o0.y += p0.y; o0.z += p0.z; o0.w += p0.w;
            o1.x += p1.x; o1.y += p1.y; o1.z += p1.z; o1.w += p1.w;
          }
          C[0] = o0;
          C[1] = o1;
        }
      } else {
        for (int e = 0; e < 8 && col + e < g.N; ++e) {
          const size_t o = (size_t)row * g.ldc + col + e;
          if (g.out_bf16) {
            uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
            C[o] = (uint16_t)f32_to_bf16_bits(v[e] + (g.accumulate ? bf2f(C[o]) : 0.f));
          } else {
            float* C = reinterpret_cast<float*>(g.C);
            C[o] = v[e] + (g.accumulate ? C[o] : 0.f);
          }
        }
      }
    }
  }
}

// Branch-free specialization of store_direct for the common case (splitk 1, no
// accumulate, no activation, 16-B aligned C, N % 8 == 0): output type and bias
// kind are compile-time, so the epilogue is straight-line code (the generic one
// unrolls every runtime combination into ~12k instructions).
template <bool OUT_BF16, int BIAS>
__device__ __forceinline__ void store_direct_fast(const GemmArgs& g, const floatx4 (&acc)[4][4], int row0, int col0,
                                                  int lane) {
  const int c = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int col = col0 + 32 * p + 8 * gq;
    float bias[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if constexpr (BIAS == 1) bias[e] = col < g.N ? reinterpret_cast<const float*>(g.bias)[col + e] : 0.f;
      else if constexpr (BIAS == 2) bias[e] = col < g.N ? bf2f(reinterpret_cast<const uint16_t*>(g.bias)[col + e]) : 0.f;
      else bias[e] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + 16 * i + c;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = g.alpha * acc[i][2 * p + (e >> 2)][e & 3] + bias[e];
      if (row < g.M && col < g.N) {
        if constexpr (OUT_BF16) {
          uint32_t w[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) w[q] = pk_bf16(v[2 * q], v[2 * q + 1]);
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(g.C) + (size_t)row * g.ldc + col) =
              uint4{w[0], w[1], w[2], w[3]};
        } else {
          float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col);
          C[0] = make_float4(v[0], v[1], v[2], v[3]);
          C[1] = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
  }
}

__global__ void __launch_bounds__(NT) k_gemm_nt(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[(2 * (BM + BN) * kRowBytes > BM * (BN + 4) * 4) ? 2 * (BM + BN) * kRowBytes : BM * (BN + 4) * 4];
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m * g.splitk;
  // bijective XCD-aware remap: blocks b, b+8, b+16, ... (same XCD) get consecutive ids;
  // the K slices of one tile are adjacent ids, so they share an XCD (and its L2)
  int wg = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = wg % 8;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / 8;
  }
  const int split = wg % g.splitk;
  wg /= g.splitk;
  const int bm = (wg / tiles_n) * BM, bn = (wg % tiles_n) * BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  auto As = [&](int buf) { return smem + buf * ((BM + BN) * kRowBytes); };
  auto Bs = [&](int buf) { return smem + buf * ((BM + BN) * kRowBytes) + BM * kRowBytes; };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  const int srow = t >> 3, schunk = t & 7;
  auto gload = [&](int k0) {
    const int gk = k0 + schunk * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = srow + 32 * i;
      const int gm = bm + r, gn = bn + r;
      ra[i] = (gm < g.M && gk < g.K) ? *reinterpret_cast<const uint4*>(g.A + (size_t)gm * g.lda + gk) : uint4{0, 0, 0, 0};
      rb[i] = (gn < g.N && gk < g.K) ? *reinterpret_cast<const uint4*>(g.B + (size_t)gn * g.ldb + gk) : uint4{0, 0, 0, 0};
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = srow + 32 * i;
      const int off = r * kRowBytes + ((schunk ^ (r & 7)) << 4);
      *reinterpret_cast<uint4*>(As(buf) + off) = ra[i];
      *reinterpret_cast<uint4*>(Bs(buf) + off) = rb[i];
    }
  };

  const int nk_all = (g.K + BK - 1) / BK;
  const int per = (nk_all + g.splitk - 1) / g.splitk;
  const int kt0 = split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  if (nk > 0) {
    gload(kt0 * BK);
    swrite(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt0 + kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bf[4];
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra_ = wm + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As(cur) + ra_ * kRowBytes + ((chunk ^ (ra_ & 7)) << 4));
        const int rb_ = wn + i * 16 + (lane & 15);
        bf[i] = *reinterpret_cast<const bf16x8*>(Bs(cur) + rb_ * kRowBytes + ((chunk ^ (rb_ & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }

  __syncthreads();
  store_tile(g, acc, smem, bm, bn, wm, wn, split, t, lane);
}

// Same tile / wave layout as k_gemm_nt, staged by LDS-DMA (global_load_lds,
// 16 B per lane, 1 KiB per wave instruction) instead of registers: the next
// K-tile streams straight into the other LDS buffer while this one feeds the
// MFMAs, and the staging costs no VGPRs and no ds_write issue slots.  The LDS
// image is lane-linear (8 rows of 128 B per instruction), so the (row & 7)
// chunk swizzle the fragment reads expect is applied to the per-lane SOURCE
// address (the same involution on both sides).  Rows past M / N re-read the
// last valid row (their outputs are discarded); used only when K % 64 == 0.
__constant__ int g_pp_exp_dev = 0;

// DIRECT: swapped MFMA operands + pair-permuted B staging + LDS-free epilogue
// (store_direct); otherwise the LDS-staged row epilogue (store_tile).
template <bool DIRECT, int FAST = 0>  // FAST = 1 + out_bf16 + 2 * bias_kind (store_direct_fast), 0 = generic
__global__ void __launch_bounds__(NT) k_gemm_nt_glds(GemmArgs g) {
  constexpr int kLoop = 2 * (BM + BN) * kRowBytes, kEpi = DIRECT ? 0 : BM * (BN + 4) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLoop > kEpi ? kLoop : kEpi];
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m * g.splitk;
  int wg = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = wg % 8;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / 8;
  }
  const int split = wg % g.splitk;
  wg /= g.splitk;
  const int bm = (wg / tiles_n) * BM, bn = (wg % tiles_n) * BN;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  auto As = [&](int buf) { return smem + buf * ((BM + BN) * kRowBytes); };
  auto Bs = [&](int buf) { return smem + buf * ((BM + BN) * kRowBytes) + BM * kRowBytes; };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // per-lane source row / swizzled chunk for the 4 instructions of this wave
  const int lrow = lane >> 3, pchunk = lane & 7;
  auto issue = [&](int k0, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wave * 4 + i;                 // 1 KiB LDS chunk = rows q*8 .. q*8+7
      const int r = q * 8 + lrow;
      const int c = pchunk ^ (r & 7);             // logical k-chunk this lane must fetch
      const int ga = min(bm + r, g.M - 1), gb = min(bn + (DIRECT ? pair_perm(r) : r), g.N - 1);
      __builtin_amdgcn_global_load_lds((const void*)(g.A + (size_t)ga * g.lda + k0 + c * 8),
                                       (__attribute__((address_space(3))) void*)(As(buf) + q * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(g.B + (size_t)gb * g.ldb + k0 + c * 8),
                                       (__attribute__((address_space(3))) void*)(Bs(buf) + q * 1024), 16, 0, 0);
    }
  };
  const int nk_all = g.K / BK;
  const int per = (nk_all + g.splitk - 1) / g.splitk;
  const int kt0 = split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  if (nk > 0) issue(kt0 * BK, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // all fragment reads of this K-tile BEFORE the next tile's DMA is issued:
    // the compiler cannot prove the DMA target disjoint from the reads and
    // would otherwise wait for the DMA before the remaining ds_reads
    bf16x8 af[2][4], bf[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra_ = wm + i * 16 + (lane & 15);
        af[ks][i] = *reinterpret_cast<const bf16x8*>(As(cur) + ra_ * kRowBytes + ((chunk ^ (ra_ & 7)) << 4));
        const int rb_ = wn + i * 16 + (lane & 15);
        bf[ks][i] = *reinterpret_cast<const bf16x8*>(Bs(cur) + rb_ * kRowBytes + ((chunk ^ (rb_ & 7)) << 4));
      }
    }
    if (kt + 1 < nk) issue((kt0 + kt + 1) * BK, cur ^ 1);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (DIRECT) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (g_pp_exp_dev & 8) {  // ablation (benchmarks only): no epilogue, accumulators kept live
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  constexpr bool kFastBf16 = ((FAST - 1) & 1) != 0;
  constexpr int kFastBias = (FAST - 1) / 2;
  if constexpr (DIRECT && FAST > 0) store_direct_fast<kFastBf16, kFastBias>(g, acc, bm + wm, bn + wn, lane);
  else if constexpr (DIRECT) store_direct(g, acc, bm + wm, bn + wn, split, lane);
  else store_tile(g, acc, smem, bm, bn, wm, wn, split, t, lane);
}



// ---------------------------------------------------------------------------
// "TN" GEMM for weight gradients: C[N1,N2] (+)= alpha * sum_m A[m,n1] * B[m,n2]
// with A [M][N1] and B [M][N2] row-major (n contiguous), i.e. dW = dY^T X
// without materialising any transpose.  Tiles of 64 m-rows x 128 columns are
// staged as-is into LDS; MFMA operands (8 consecutive m for one column per
// lane) come out of gfx950's transposing LDS read ds_read_b64_tr_b16, two
// reads per operand per 32-deep k-step.  LDS rows are 256 B + 32 B pad (row r
// starts 8 banks after row r-1) and the two 128-B halves of rows with bit 3
// set are swapped, so every tr read (a 32-lane half spans rows r..r+3 and
// r+8..r+11) is bank-conflict free.  K (= batch*seq) is long and M, N small:
// the split-K grid fills the chip and partial tiles meet through fp32
// atomic adds.
// ---------------------------------------------------------------------------
typedef short v4s __attribute__((ext_vector_type(4)));
constexpr int kTnRow = 288;             // bytes per LDS row (256 data + 32 pad)
constexpr int kTnTile = BK * kTnRow;    // one operand tile

__device__ __forceinline__ int tn_off(int row, int byte) { return row * kTnRow + (byte ^ (((row >> 3) & 1) << 7)); }

// FAST: 0 generic store_tile, 1 split-K atomics, 2 plain stores, 3 accumulating stores,
// 4 split-K partial into a workspace slice (fp32 C, 16-B aligned, N2 % 4 == 0).
// split_major = 1: logical id = split * tiles + tile, so after the XCD remap one XCD
// runs every output tile of a few consecutive K slices: the K slice's rows of A
// and B are fetched into that XCD's L2 once and shared by all its tiles (with
// split-minor order each XCD streams whole K panels of its own few tiles, and
// the same bytes cross the fabric once per tile).
// PF: K tiles in flight per workgroup.  PF = 1 issues tile k+1's global loads under tile k's
// MFMAs; PF = 2 keeps tiles k+1 and k+2 in flight in two register sets (the loop unrolled so
// the sets are indexed statically): 5-8 % faster on the dQKV^T Xp and 4096^2 shapes.  PF = 4
// (one wave per SIMD) measured no faster on the narrow shape and 20 % slower on the wide ones
// (profiles/r5_train_kernels/gemm_tn_pf4.jsonl), so only 1 and 2 are built.
template <int FAST, int PF = 1>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PF >= 4 ? 1 : 2))) k_gemm_tn(GemmArgs g, int split_major) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * kTnTile];
  // here: g.M = N1 (rows of C), g.N = N2 (cols of C), g.K = M (reduction)
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m * g.splitk;
  int wg = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = wg % 8;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / 8;
  }
  int split;
  if (split_major) {
    split = wg / (tiles_n * tiles_m);
    wg %= tiles_n * tiles_m;
  } else {
    split = wg % g.splitk;
    wg /= g.splitk;
  }
  const int bm = (wg / tiles_n) * BM, bn = (wg % tiles_n) * BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  auto As = [&](int buf) { return smem + buf * (2 * kTnTile); };
  auto Bs = [&](int buf) { return smem + buf * (2 * kTnTile) + kTnTile; };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[PF][4], rb[PF][4];
  const int schunk = t & 15, srow = t >> 4;  // 16 chunks of 16 B per 128-column row
  const int nk_all = (g.K + BK - 1) / BK;
  const int per = (nk_all + g.splitk - 1) / g.splitk;
  const int kt0 = split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  // PF = 2 loads through buffer resources over this split's rows: rows past K read as 0
  // with no branch, so the loads carry no exec-mask control flow and the compiler can
  // wait for the older register set alone (with the guarded pointer loads below it
  // emits vmcnt(0), draining the newer set too).  Columns past N1 / N2 read the row's
  // neighbours, which only reach outputs that are never stored.
  const int rows = max(0, min(g.K - kt0 * BK, nk * BK));
  Rsrc rsa{}, rsb{};
  if constexpr (PF >= 2) {
    rsa = make_rsrc(uniform_ptr(reinterpret_cast<char*>(const_cast<uint16_t*>(g.A + (size_t)kt0 * BK * g.lda))),
                    (uint32_t)((size_t)rows * g.lda * 2));
    rsb = make_rsrc(uniform_ptr(reinterpret_cast<char*>(const_cast<uint16_t*>(g.B + (size_t)kt0 * BK * g.ldb))),
                    (uint32_t)((size_t)rows * g.ldb * 2));
  }
  auto gload = [&](int s, int m0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + srow + 16 * i;
      const int ca = bm + schunk * 8, cb = bn + schunk * 8;
      if constexpr (PF >= 2) {
        const uint32_t ml = (uint32_t)(m - kt0 * BK);
        ra[s][i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsa.r, (ml * g.lda + ca) * 2, 0, 0));
        rb[s][i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsb.r, (ml * g.ldb + cb) * 2, 0, 0));
      } else {
        ra[s][i] = (m < g.K && ca < g.M) ? *reinterpret_cast<const uint4*>(g.A + (size_t)m * g.lda + ca) : uint4{0, 0, 0, 0};
        rb[s][i] = (m < g.K && cb < g.N) ? *reinterpret_cast<const uint4*>(g.B + (size_t)m * g.ldb + cb) : uint4{0, 0, 0, 0};
      }
    }
  };
  auto swrite = [&](int buf, int s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = srow + 16 * i;
      *reinterpret_cast<uint4*>(As(buf) + tn_off(r, schunk * 16)) = ra[s][i];
      *reinterpret_cast<uint4*>(Bs(buf) + tn_off(r, schunk * 16)) = rb[s][i];
    }
  };
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  // fragment read addresses: tn_off(ks * 32 + grp * 8 + q + 4 h, (w + 16 i + 4 p) * 2) is a
  // per-lane base plus the constant ks * 32 * kTnRow + h * 4 * kTnRow + 32 i: the half-swap
  // XOR only flips the 128-B bit that w * 2 (w in {0, 64}) owns (row bit 3 = grp & 1; q + 4h
  // < 8 never carries into it), so every read is base + an immediate offset
  const int lrow = (grp * 8 + q) * kTnRow, xsw = (grp & 1) << 7;
  const int la = lrow + ((wm * 2) ^ xsw) + 8 * p, lb = lrow + ((wn * 2) ^ xsw) + 8 * p;
  auto compute = [&](int cur) {
    const unsigned char* abase = As(cur) + la;
    const unsigned char* bbase = Bs(cur) + lb;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v4s a0, a1, b0, b1;
        const int o = ks * 32 * kTnRow + 32 * i;
        a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(abase + o));
        a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(abase + o + 4 * kTnRow));
        b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(bbase + o));
        b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(bbase + o + 4 * kTnRow));
        typedef short v8s __attribute__((ext_vector_type(8)));
        v8s av = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
        v8s bv = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
        af[i] = __builtin_bit_cast(bf16x8, av);
        bf[i] = __builtin_bit_cast(bf16x8, bv);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (PF == 1) {
    if (nk > 0) {
      gload(0, kt0 * BK);
      swrite(0, 0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(0, (kt0 + kt + 1) * BK);
      compute(cur);
      if (kt + 1 < nk) swrite(cur ^ 1, 0);
      __syncthreads();
    }
  } else {
    // tile j is loaded into register set j % PF and written to LDS buffer j & 1 one step
    // before its MFMAs; set j % PF is refilled with tile j + PF right after that write
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (u < nk) gload(u, (kt0 + u) * BK);
    if (nk > 0) swrite(0, 0);
    __syncthreads();
    if (PF < nk) gload(0, (kt0 + PF) * BK);
    for (int kt = 0; kt < nk; kt += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        if (kt + u < nk) {
          compute(u & 1);
          if (kt + u + 1 < nk) swrite((u + 1) & 1, (u + 1) % PF);
          __syncthreads();
          if (kt + u + 1 + PF < nk) gload((u + 1) % PF, (kt0 + kt + u + 1 + PF) * BK);
        }
      }
    }
  }
  __syncthreads();
  if constexpr (FAST == 1) store_tile_f32<true, false>(g, acc, smem, bm, bn, wm, wn, t, lane);
  else if constexpr (FAST == 4) {  // split-K partial -> workspace slice [split][N1][N2] (plain stores)
    GemmArgs w = g;
    w.C = reinterpret_cast<float*>(g.C) + (size_t)split * g.M * g.N;
    w.ldc = g.N;
    store_tile_f32<false, false>(w, acc, smem, bm, bn, wm, wn, t, lane);
  } else if constexpr (FAST == 2) store_tile_f32<false, false>(g, acc, smem, bm, bn, wm, wn, t, lane);
  else if constexpr (FAST == 3) store_tile_f32<false, true>(g, acc, smem, bm, bn, wm, wn, t, lane);
  else store_tile(g, acc, smem, bm, bn, wm, wn, split, t, lane);
}


// ---------------------------------------------------------------------------
// Small-K "NT" GEMM (K <= 128, e.g. the K = 72 patch embedding): the output
// write dominates, so the kernel is built around it.  Each 256-thread block
// owns a 256-column slice of B, kept in LDS for the whole launch, and walks
// 64-row tiles of A (grid-strided), prefetching the next A tile into
// registers while the current one is multiplied.  The MFMA operands are
// swapped (first = B rows, second = A rows), so the accumulator of a 16x16
// tile holds C[m = lane & 15][tile row 4*(lane >> 4) + r]; the tile rows of a
// PAIR of tiles are mapped to 32 output columns as n = 8*(i >> 2) + 4*half +
// (i & 3), so each lane ends up with 8 consecutive columns of one row and
// stores them as one 16-B (bf16) vector -- no LDS round trip, no narrow
// stores.  LDS rows are padded to an odd number of 16-B slots so 16-row
// fragment reads are conflict-free.
// ---------------------------------------------------------------------------
constexpr int SK_BM = 64, SK_NT = 256;
int g_sk_bn = std::getenv("CCMPI_SK_BN") ? std::atoi(std::getenv("CCMPI_SK_BN")) : 128;      // tuning knobs
// grid cap; 0 = one balanced round (below)
int g_sk_grid = std::getenv("CCMPI_SK_GRID") ? std::atoi(std::getenv("CCMPI_SK_GRID")) : 0;
bool g_sk_nt = std::getenv("CCMPI_SK_NT") != nullptr;  // non-temporal bf16 stores (A/B knob)

int device_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

// Patch source for the fused embedding (PATCH = true): the A rows are generated
// from the fp32 images instead of read -- token row m = (image m / S, patch m % S)
// holds the patch's p*p pixels, a constant 1 (bias column) and a one-hot patch
// position, exactly like k_patchify (attn_small.hip) -- and the blocks of the
// first N slice also store those rows to xp (the backward's copy of the input).
struct PatchSrc {
  const float* x;   // [B][img*img]
  int img, p;
  uint16_t* xp;     // [M][ld_xp] bf16 (may be null)
  int ld_xp;
};

__device__ __forceinline__ uint4 patch_chunk(const PatchSrc& ps, int m, int ch) {
  const int gp = ps.img / ps.p, S = gp * gp, pp = ps.p * ps.p;
  const int s = m % S;
  const float* xb = ps.x + (size_t)(m / S) * ps.img * ps.img + (s / gp) * ps.p * ps.img + (s % gp) * ps.p;
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v2[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int cc = ch * 8 + 2 * q + hh;
      float v = 0.f;
      if (cc < pp) v = xb[(cc / ps.p) * ps.img + cc % ps.p];
      else if (cc == pp || cc == pp + 1 + s) v = 1.f;
      v2[hh] = v;
    }
    w[q] = pk_bf16(v2[0], v2[1]);
  }
  return uint4{w[0], w[1], w[2], w[3]};
}

// LDS row of the small-K kernel: the K / 8 data chunks (16 B), plus one spare chunk when
// K is not a multiple of 32, rounded up to a chunk count u with u % 4 == 2, so the 16
// consecutive rows of a fragment read (lane groups of ds_read_b128) land on 16 distinct
// 4-bank groups.  Reads of chunks past K go to ONE zero chunk (B row 0's spare chunk,
// a broadcast) instead of zero-padded row columns.  Measured: the former rows of
// round_up(K, 32) + 8 elements had 44 % of LDS cycles in bank conflicts
// (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) and room for 3 workgroups per CU, not 4.
__host__ __device__ inline int sk_row_chunks(int K) {
  int u = K / 8 + (K % 32 ? 1 : 0);
  while (u % 4 != 2) ++u;
  return u;
}
inline size_t sk_lds_bytes(int skbn, int K) { return (size_t)(skbn + 2 * SK_BM) * sk_row_chunks(K) * 16; }

template <int SK_BN, int FAST = 0, bool PATCH = false>  // FAST = 1 + out_bf16 (no accumulate / act, aligned C, N % 8 == 0), 0 = generic; 3 = bf16 non-temporal
__global__ void __launch_bounds__(SK_NT) k_gemm_smallk(GemmArgs g, int kp, PatchSrc ps) {
  constexpr int WN = SK_BN / 4;  // columns per wave
  constexpr int NP = WN / 32;    // column pairs (32 columns) per wave
  constexpr int NJ = 2 * NP;     // 16-col MFMA tiles per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char sks[];
  const int stride = sk_row_chunks(g.K) * 16;       // bytes per LDS row
  unsigned char* Bs = sks;                          // SK_BN rows (fragment-order permuted, below)
  unsigned char* As = sks + SK_BN * stride;         // 2 x SK_BM rows
  const unsigned char* zchunk = sks + (g.K / 8) * 16;  // B row 0's spare chunk: 16 zero bytes
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, c = lane & 15, gq = lane >> 4;
  const int kchunks = g.K / 8;                      // 16-B data chunks per row
  const int tiles_n = (g.N + SK_BN - 1) / SK_BN, tiles_m = (g.M + SK_BM - 1) / SK_BM;
  const int tn = blockIdx.x % tiles_n;
  const int bn = tn * SK_BN;
  const int mstep = gridDim.x / tiles_n;            // blocks sharing this N slice
  int tm = blockIdx.x / tiles_n;
  if (tm >= tiles_m) return;
  if (t == 0) *reinterpret_cast<uint4*>(const_cast<unsigned char*>(zchunk)) = uint4{0, 0, 0, 0};
  // B slice -> LDS (zero rows past N).  Slice row r = 32p + 8*(c >> 2) + 4h + (c & 3) feeds
  // MFMA row c of tile j = 2p + h (the column permutation described above); it is stored
  // at LDS row 32p + 16h + c, so a tile's 16 fragment rows are 16 consecutive LDS rows,
  // read as conflict-free as the A rows.
  for (int idx = t; idx < SK_BN * kchunks; idx += SK_NT) {
    const int r = idx / kchunks, ch = idx % kchunks;
    const int rl = r & 31, pos = (r & ~31) | (((rl >> 2) & 1) << 4) | ((rl >> 3) << 2) | (rl & 3);
    uint4 v{0, 0, 0, 0};
    if (bn + r < g.N) v = *reinterpret_cast<const uint4*>(g.B + (size_t)(bn + r) * g.ldb + ch * 8);
    *reinterpret_cast<uint4*>(Bs + pos * stride + ch * 16) = v;
  }
  constexpr int kMaxPer = SK_BM * 16 / SK_NT;       // A chunks per thread at K = 128
  uint4 ra[kMaxPer];
  const int per = (SK_BM * kchunks + SK_NT - 1) / SK_NT;
  auto gload = [&](int m0) {
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i) {
      const int idx = t + i * SK_NT, r = idx / kchunks, ch = idx % kchunks;
      ra[i] = uint4{0, 0, 0, 0};
      if (i < per && r < SK_BM && m0 + r < g.M) {
        if constexpr (PATCH) {
          ra[i] = patch_chunk(ps, m0 + r, ch);
          if (tn == 0 && ps.xp) *reinterpret_cast<uint4*>(ps.xp + (size_t)(m0 + r) * ps.ld_xp + ch * 8) = ra[i];
        } else {
          ra[i] = *reinterpret_cast<const uint4*>(g.A + (size_t)(m0 + r) * g.lda + ch * 8);
        }
      }
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i) {
      const int idx = t + i * SK_NT, r = idx / kchunks, ch = idx % kchunks;
      if (i < per && r < SK_BM) *reinterpret_cast<uint4*>(As + (buf * SK_BM + r) * stride + ch * 16) = ra[i];
    }
  };
  gload(tm * SK_BM);
  swrite(0);
  __syncthreads();
  // this lane's output columns: pair p (32 columns) -> bn + WN*wave + 32p + 8*gq + 0..7
  float bias[NP][8];
#pragma unroll
  for (int pr = 0; pr < NP; ++pr)
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[pr][e] = load_bias(g, bn + wave * WN + pr * 32 + 8 * gq + e, 0);
  const int es = g.out_bf16 ? 2 : 4;
  const bool vec_ok = (((uint64_t)g.C | ((uint64_t)g.ldc * es)) % 16) == 0;
  int buf = 0;
  for (; tm < tiles_m; tm += mstep) {
    const int m0 = tm * SK_BM;
    const bool more = tm + mstep < tiles_m;
    if (more) gload((tm + mstep) * SK_BM);
    floatx4 acc[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const unsigned char* A = As + buf * SK_BM * stride;
    for (int ks = 0; ks < kp / 32; ++ks) {
      const int ch = 4 * ks + gq;
      const bool z = ch >= kchunks;  // past K: the shared zero chunk
      bf16x8 fb[NJ], fa[4];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(z ? zchunk : Bs + (wave * WN + 16 * j + c) * stride + ch * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(z ? zchunk : A + (i * 16 + c) * stride + ch * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    // epilogue: lane holds C[m0 + 16i + c][bn + WN*wave + 32p + 8*gq + e], e = 4*half + r
    if constexpr (FAST > 0) {  // straight-line: one 16-B (bf16) / 2 x 16-B (fp32) store per row and pair
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + i * 16 + c;
#pragma unroll
        for (int pr = 0; pr < NP; ++pr) {
          const int col = bn + wave * WN + pr * 32 + 8 * gq;
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = g.alpha * acc[i][2 * pr + (e >> 2)][e & 3] + bias[pr][e];
          if (row < g.M && col < g.N) {
            if constexpr (FAST >= 2) {
              uint32_t w[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) w[q] = pk_bf16(v[2 * q], v[2 * q + 1]);
              uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(g.C) + (size_t)row * g.ldc + col);
              if constexpr (FAST == 3) {  // streaming (non-temporal) store: A/B knob for the write-bound case
                typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(u32x4v{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4v*>(dst));
              } else {
                *dst = uint4{w[0], w[1], w[2], w[3]};
              }
            } else {
              float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col);
              C[0] = make_float4(v[0], v[1], v[2], v[3]);
              C[1] = make_float4(v[4], v[5], v[6], v[7]);
            }
          }
        }
      }
    } else
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + i * 16 + c;
      if (row >= g.M) continue;
#pragma unroll
      for (int pr = 0; pr < NP; ++pr) {
        const int col = bn + wave * WN + pr * 32 + 8 * gq;
        if (col >= g.N) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = epi(g, acc[i][2 * pr + (e >> 2)][e & 3], bias[pr][e]);
        if (vec_ok && col + 8 <= g.N) {
          if (g.out_bf16) {
            uint16_t* C = reinterpret_cast<uint16_t*>(g.C) + (size_t)row * g.ldc + col;
            if (g.accumulate) {
              const uint4 o = *reinterpret_cast<const uint4*>(C);
              const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
              for (int q = 0; q < 4; ++q) { v[2 * q] += bf16_lo(ow[q]); v[2 * q + 1] += bf16_hi(ow[q]); }
            }
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) w[q] = pk_bf16(v[2 * q], v[2 * q + 1]);
            *reinterpret_cast<uint4*>(C) = uint4{w[0], w[1], w[2], w[3]};
          } else {
            float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col);
            float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
            if (g.accumulate) {
              const float4 p0 = C[0], p1 = C[1];
              o0.x += p0.x; o0.y += p0.y; o0.z += p0.z; o0.w += p0.w;
              o1.x += p1.x; o1.y += p1.y; o1.z += p1.z; o1.w += p1.w;
            }
            C[0] = o0;
            C[1] = o1;
          }
        } else {
          for (int e = 0; e < 8 && col + e < g.N; ++e) {
            const size_t o = (size_t)row * g.ldc + col + e;
            if (g.out_bf16) {
              uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
              C[o] = (uint16_t)f32_to_bf16_bits(v[e] + (g.accumulate ? bf2f(C[o]) : 0.f));
            } else {
              float* C = reinterpret_cast<float*>(g.C);
              C[o] = v[e] + (g.accumulate ? C[o] : 0.f);
            }
          }
        }
      }
    }
    if (more) swrite(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
}

// 2-D transpose of 16-bit elements through a padded 64x65 LDS tile.
__global__ void __launch_bounds__(256) k_transpose16(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                     int R, int C, int lds, int ldd) {
  __shared__ uint16_t tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int y = ty; y < 64; y += 4) {
    const int r = r0 + y, c = c0 + tx;
    if (r < R && c < C) tile[y][tx] = src[(size_t)r * lds + c];
  }
  __syncthreads();
  for (int y = ty; y < 64; y += 4) {
    const int c = c0 + y, r = r0 + tx;  // dst row = c, col = r
    if (c < C && r < R) dst[(size_t)c * ldd + r] = tile[tx][y];
  }
}

// The same with 16-B accesses and no LDS: lane l of wave w takes an 8-row x 16-column
// block (rows r0 + 8 l .., columns c0 + 16 w ..; 8 x 2 row loads of 16 B), transposes its
// two 8 x 8 halves in registers and writes 16 destination rows of 16 B.  A workgroup covers
// 512 x 64: each source row's 128-B line is read whole by its four waves, every store
// instruction writes 1 KiB of consecutive bytes.  R, C, strides % 8 == 0, 16-B aligned.
__global__ void __launch_bounds__(256) k_transpose16_v(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                       int R, int C, int lds, int ldd) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.y * 512 + 8 * lane, c = blockIdx.x * 64 + 16 * wave;
  if (r >= R) return;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int cb = c + 8 * b;
    if (cb >= C) break;
    uint4 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = *reinterpret_cast<const uint4*>(src + (size_t)(r + i) * lds + cb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t o[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const uint4& x = q[2 * m];
        const uint4& y = q[2 * m + 1];
        const uint32_t xw = (j >> 1) == 0 ? x.x : (j >> 1) == 1 ? x.y : (j >> 1) == 2 ? x.z : x.w;
        const uint32_t yw = (j >> 1) == 0 ? y.x : (j >> 1) == 1 ? y.y : (j >> 1) == 2 ? y.z : y.w;
        o[m] = (j & 1) ? ((xw >> 16) | (yw & 0xffff0000u)) : ((xw & 0xffffu) | (yw << 16));
      }
      *reinterpret_cast<uint4*>(dst + (size_t)(cb + j) * ldd + r) = uint4{o[0], o[1], o[2], o[3]};
    }
  }
}

// LDS variant: a workgroup moves a 64 x 64 tile.  Loads: 8 lanes per source row, 16 B
// each (a wave reads 8 whole 128-B lines); the tile lands in LDS with a 33-word row
// stride (odd: the column gathers below are bank-conflict free).  Stores: 8 lanes per
// destination row, each packing 8 source rows of one column (8 ds_read_u16) into 16 B.
__global__ void __launch_bounds__(256) k_transpose16_l(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                       int R, int C, int lds, int ldd) {
  constexpr int S = 66;  // row stride in elements (33 words)
  __shared__ uint32_t tile[64 * S / 2];
  const int t = threadIdx.x;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int lr = t >> 3, lc = (t & 7) * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = lr + 32 * h;
    uint4 v = uint4{0u, 0u, 0u, 0u};
    if (r0 + row < R && c0 + lc < C) v = *reinterpret_cast<const uint4*>(src + (size_t)(r0 + row) * lds + c0 + lc);
    uint32_t* d = tile + (row * S + lc) / 2;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int oc = lr + 32 * h, q = t & 7;  // destination row c0 + oc, source rows 8 q ..
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
      o[m] = (uint32_t)t16[(8 * q + 2 * m) * S + oc] | ((uint32_t)t16[(8 * q + 2 * m + 1) * S + oc] << 16);
    if (c0 + oc < C && r0 + 8 * q < R)
      *reinterpret_cast<uint4*>(dst + (size_t)(c0 + oc) * ldd + r0 + 8 * q) = uint4{o[0], o[1], o[2], o[3]};
  }
}

// Sum of the split-K workspace slices into C ([rows][cols] fp32, row stride ldc),
// 4 columns per thread: C (+)= sum_s ws[s].  Columns >= csplit (a multiple of 4)
// go to a second destination instead, C2[r][c - csplit] = sum (overwritten):
// one GEMM over a row-concatenated operand [X | Y] yields A^T X accumulated
// into one buffer and A^T Y into another, with no copy pass.
__global__ void __launch_bounds__(256) k_splitk_reduce(const float* __restrict__ ws, int splitk, float* __restrict__ C,
                                                       int ldc, int rows, int cols, int accumulate,
                                                       float* __restrict__ C2, int ldc2, int csplit) {
  const size_t slice = (size_t)rows * cols;
  const int vc = cols / 4;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)rows * vc; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / vc), c = (int)(e % vc) * 4;
    const float* src = ws + (size_t)r * cols + c;
    float4 acc = *reinterpret_cast<const float4*>(src);
    for (int k = 1; k < splitk; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(src + k * slice);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (c >= csplit) {
      *reinterpret_cast<float4*>(C2 + (size_t)r * ldc2 + (c - csplit)) = acc;
      continue;
    }
    float4* dst = reinterpret_cast<float4*>(C + (size_t)r * ldc + c);
    if (accumulate) {
      const float4 o = *dst;
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
    }
    *dst = acc;
  }
}

// Small-K launcher (patch embedding, K <= 96): B slice resident in LDS, A tiles streamed
// (or generated from the images, PATCH), direct stores.  id = FAST variant (0 generic,
// 1 fp32 out, 2 bf16 out); patch sources need id 2.
void launch_smallk(const GemmArgs& g, int id, const PatchSrc& ps, hipStream_t st) {
  const int kp = (g.K + 31) / 32 * 32;
  const int skbn = (g_sk_bn == 256 && !ps.x) ? 256 : 128;
  const int tiles_n = (g.N + skbn - 1) / skbn, tiles_m = (g.M + SK_BM - 1) / SK_BM;
  const size_t lds = sk_lds_bytes(skbn, g.K);
  // Every block loads its B slice once, then walks M tiles: the grid is one round of
  // resident blocks (LDS-limited per CU) with the same number of M tiles in every block
  // (an uneven split leaves half the blocks idle for the last tile).  Measured on the
  // 32768 x 768 x 72 embedding: 3 blocks per CU, 768 blocks x 4 tiles: 23.6 us; a
  // 2048-block grid (1-2 tiles each): 28-29 us (benchmarks/emb_write_probe.py).
  int mblocks;
  if (g_sk_grid > 0) {
    mblocks = std::max(1, std::min(tiles_m, std::max(1, g_sk_grid / tiles_n)));
  } else {
    const int per_cu = std::max(1, (int)((160u * 1024u) / lds));
    const int cap = std::max(1, per_cu * device_cus() / tiles_n);   // resident blocks per N slice
    const int rounds = (tiles_m + cap - 1) / cap;                    // M tiles per block
    mblocks = (tiles_m + rounds - 1) / rounds;
  }
  static bool attr = [] {
    bool ok = true;
    for (const void* f : {reinterpret_cast<const void*>(k_gemm_smallk<256, 0>),
                          reinterpret_cast<const void*>(k_gemm_smallk<128, 0>),
                          reinterpret_cast<const void*>(k_gemm_smallk<128, 1>),
                          reinterpret_cast<const void*>(k_gemm_smallk<128, 2>),
                          reinterpret_cast<const void*>(k_gemm_smallk<128, 3>),
                          reinterpret_cast<const void*>(k_gemm_smallk<128, 2, true>)})
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
  }();
  (void)attr;
  const dim3 grid(tiles_n * mblocks);
  if (ps.x) {
    if (id != 2) throw std::invalid_argument("ccmpi: the fused patch embedding needs the bf16 fast epilogue");
    hipLaunchKernelGGL((k_gemm_smallk<128, 2, true>), grid, dim3(SK_NT), lds, st, g, kp, ps);
  } else if (skbn == 256) {
    hipLaunchKernelGGL((k_gemm_smallk<256, 0>), grid, dim3(SK_NT), lds, st, g, kp, ps);
  } else if (id == 1) {
    hipLaunchKernelGGL((k_gemm_smallk<128, 1>), grid, dim3(SK_NT), lds, st, g, kp, ps);
  } else if (id == 2) {
    if (g_sk_nt) hipLaunchKernelGGL((k_gemm_smallk<128, 3>), grid, dim3(SK_NT), lds, st, g, kp, ps);
    else hipLaunchKernelGGL((k_gemm_smallk<128, 2>), grid, dim3(SK_NT), lds, st, g, kp, ps);
  } else {
    hipLaunchKernelGGL((k_gemm_smallk<128, 0>), grid, dim3(SK_NT), lds, st, g, kp, ps);
  }
  CCMPI_HIP_CHECK(hipGetLastError());
}

// Fused MNIST patch embedding: h[M][N] = patches(x)[M][K] . W[N][K]^T, bf16 out, with the
// patch rows (pixels | 1 | one-hot position | 0 pad, K = kp of the model) generated from
// the fp32 images inside the GEMM and also stored to xp (row stride ld_xp) for the backward.
void embed_patches(uint64_t x, uint64_t W, uint64_t C, int B, int img, int p, int N, int K, int ldw, int ldc,
                   uint64_t xp, int ld_xp, uint64_t stream) {
  const int S = (img / p) * (img / p), M = B * S;
  if (M <= 0 || N <= 0) return;
  if (K % 8 || K > 96 || K < p * p + 1 + S || ldw % 8 || ldc % 8 || N % 8 || (W % 16) || (C % 16) ||
      (xp && (ld_xp % 8 || (xp % 16))) || M < 4 * SK_BM)
    throw std::invalid_argument("ccmpi embed_patches: K % 8 == 0, p*p + 1 + S <= K <= 96, 16-B aligned rows, N % 8 == 0");
  GemmArgs g{nullptr, reinterpret_cast<const uint16_t*>(W), reinterpret_cast<void*>(C), nullptr, M, N, K, K, ldw, ldc,
             1.f, 0, 0, 0, 1, 1};
  launch_smallk(g, 2, PatchSrc{reinterpret_cast<const float*>(x), img, p, reinterpret_cast<uint16_t*>(xp), ld_xp},
                reinterpret_cast<hipStream_t>(stream));
}

void gemm_nt(uint64_t A, uint64_t B, uint64_t C, uint64_t bias, int M, int N, int K, int lda, int ldb, int ldc,
             float alpha, bool accumulate, int bias_kind, int act, bool out_bf16, int splitk, uint64_t stream) {
  if (M <= 0 || N <= 0) return;
  if (K % 8 || lda % 8 || ldb % 8 || (A % 16) || (B % 16))
    throw std::invalid_argument("ccmpi gemm: K, lda, ldb must be multiples of 8 and A/B 16-B aligned");
  if (splitk < 1) splitk = 1;
  if (splitk > 1 && (out_bf16 || act != 0))
    throw std::invalid_argument("ccmpi gemm: split-K needs an fp32 output and no activation");
  if (splitk > 1 && !accumulate)
    CCMPI_HIP_CHECK(hipMemset2DAsync(reinterpret_cast<void*>(C), (size_t)ldc * 4, 0, (size_t)N * 4, M,
                                     reinterpret_cast<hipStream_t>(stream)));
  GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B), reinterpret_cast<void*>(C),
             reinterpret_cast<const void*>(bias), M, N, K, lda, ldb, ldc, alpha, accumulate ? 1 : 0, bias_kind,
             act, out_bf16 ? 1 : 0, splitk};
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN) * splitk;
  // small K (patch embedding): B slice resident in LDS, A tiles streamed, direct stores
  // measured (benchmarks/smallk_sweep.py): wins over the 128x128 kernel up to K ~ 96
  if (K <= 96 && splitk == 1 && g_kernel != 1 && g_sk_bn > 0 && M >= 4 * SK_BM) {
    const bool fast = !accumulate && act == 0 && N % 8 == 0 && ldc % 8 == 0 && (C % 16) == 0;
    launch_smallk(g, fast ? 1 + (out_bf16 ? 1 : 0) : 0, PatchSrc{}, reinterpret_cast<hipStream_t>(stream));
    return;
  }
  // 256 x {256, 192, 128} ping-pong kernels: need K % 128 and enough tiles to
  // occupy the 256 CUs (one block per CU); smaller grids keep 128x128.
  if (g_kernel == 5 && gemm_w4_ok(g)) {
    launch_gemm_nt_w4(g, reinterpret_cast<hipStream_t>(stream));
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  // auto: large bf16-out GEMMs on the four-wave LDS-ring kernel (gemm_w4.hip; measured
  // against the 256x256 ping-pong kernel in profiles/r3_gemm)
  // (long K over at most one tile per CU stays on the 256x256 ping-pong kernel: 4096^2 x
  // 28672 measured 1291-1368 TF/s there against 1224-1252 on the ring; ring sched bit 15
  // sends it to the ring too)
  if (g_kernel == 0 && splitk == 1 && g_ring_min_macs > 0 && (long long)M * N * K >= g_ring_min_macs &&
      M >= 1024 && N >= 1024 && ((g_ring_sched & 32768) || !(K > 16384 && gemm_w4_tiles(M, N) <= 256)) &&
      gemm_w4_ok(g) && gemm_w4r_fast(g)) {
    launch_gemm_nt_w4r(g, reinterpret_cast<hipStream_t>(stream));
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  const bool big_ok = K % (2 * BK) == 0 && g_use_glds;
  if (big_ok && g_kernel != 1) {
    int bn = 0;
    if (g_kernel == 2) bn = 256;
    else if (g_kernel == 3) bn = 128;
    else if (g_kernel == 4) bn = 192;
    // measured (benchmarks/gemm_bench.py, profiles/r1_gemm_fastepi): with the branch-free
    // epilogues the 128x128 kernel matches 256x256 up to ~256 tiles and for short K;
    // 256x256 wins with >= 2 tiles per CU and K >= 1024
    else if (gemm256_tiles(M, N, 256) * splitk >= 512 && K >= 1024 && M >= 1024 && N >= 1024) bn = 256;
    // the long-K case the ring kernel leaves to this one (above): 4096^2 x 28672 ran 0.99 ms
    // on the 128x128 kernel against 0.75 ms here (profiles/r3_swiglu/gemm_sweep.txt)
    else if (splitk == 1 && K > 16384 && M >= 1024 && N >= 1024 && gemm_w4_tiles(M, N) <= 256) bn = 256;
    if (bn) {
      launch_gemm_nt_256(g, bn, reinterpret_cast<hipStream_t>(stream));
      CCMPI_HIP_CHECK(hipGetLastError());
      return;
    }
  }
  if (K % BK == 0 && g_use_glds) {
    if (g_direct_epi) {
      const bool fast = splitk == 1 && !accumulate && act == 0 && N % 8 == 0 && ldc % 8 == 0 && (C % 16) == 0;
      const int id = fast ? 1 + (out_bf16 ? 1 : 0) + 2 * bias_kind : 0;
      auto st = reinterpret_cast<hipStream_t>(stream);
      switch (id) {
        case 1: hipLaunchKernelGGL((k_gemm_nt_glds<true, 1>), dim3(nwg), dim3(NT), 0, st, g); break;
        case 2: hipLaunchKernelGGL((k_gemm_nt_glds<true, 2>), dim3(nwg), dim3(NT), 0, st, g); break;
        case 3: hipLaunchKernelGGL((k_gemm_nt_glds<true, 3>), dim3(nwg), dim3(NT), 0, st, g); break;
        case 4: hipLaunchKernelGGL((k_gemm_nt_glds<true, 4>), dim3(nwg), dim3(NT), 0, st, g); break;
        case 5: hipLaunchKernelGGL((k_gemm_nt_glds<true, 5>), dim3(nwg), dim3(NT), 0, st, g); break;
        case 6: hipLaunchKernelGGL((k_gemm_nt_glds<true, 6>), dim3(nwg), dim3(NT), 0, st, g); break;
        default: hipLaunchKernelGGL((k_gemm_nt_glds<true, 0>), dim3(nwg), dim3(NT), 0, st, g); break;
      }
    }
    else
      hipLaunchKernelGGL(k_gemm_nt_glds<false>, dim3(nwg), dim3(NT), 0, reinterpret_cast<hipStream_t>(stream), g);
  }
  else
    hipLaunchKernelGGL(k_gemm_nt, dim3(nwg), dim3(NT), 0, reinterpret_cast<hipStream_t>(stream), g);
  CCMPI_HIP_CHECK(hipGetLastError());
}


// LDS-ring GEMM with operand layouts (gemm_w4.hip): C[M,N] (+)= alpha * op(A) op(B)^T,
// op(A)[m][k] = ta ? A[k*lda + m] : A[m*lda + k], op(B)[n][k] likewise.  Returns false
// (nothing launched) when the ring kernel does not apply (K % 64, alignment, 2 GiB).
bool gemm_ring(uint64_t A, uint64_t B, uint64_t C, int M, int N, int K, int lda, int ldb, int ldc, int ta, int tb,
               float alpha, bool accumulate, bool out_bf16, uint64_t stream) {
  if (M <= 0 || N <= 0) return true;
  GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B), reinterpret_cast<void*>(C),
             nullptr, M, N, K, lda, ldb, ldc, alpha, accumulate ? 1 : 0, 0, 0, out_bf16 ? 1 : 0, 1};
  if (!gemm_ring_ok(g, ta, tb) || (C % 16) || ldc % 8) return false;
  launch_gemm_ring(g, ta, tb, reinterpret_cast<hipStream_t>(stream));
  CCMPI_HIP_CHECK(hipGetLastError());
  return true;
}

int g_tn_split_major = std::getenv("CCMPI_TN_ORDER") ? std::atoi(std::getenv("CCMPI_TN_ORDER")) : 1;
// K tiles in flight in the 128x128 TN kernel: 0 = auto (two when a split walks >= 4 tiles), 1, 2
int g_tn_pf = std::getenv("CCMPI_TN_PF") ? std::atoi(std::getenv("CCMPI_TN_PF")) : 0;

// C[N1,N2] (+)= alpha * A[M,N1]^T . B[M,N2]; fp32 output.
void gemm_tn(uint64_t A, uint64_t B, uint64_t C, int M, int N1, int N2, int lda, int ldb, int ldc, float alpha,
             bool accumulate, int splitk, uint64_t stream, uint64_t workspace, int variant, uint64_t C2, int ldc2,
             int csplit) {
  if (N1 <= 0 || N2 <= 0 || M <= 0) return;
  if (csplit <= 0 || csplit >= N2) {
    csplit = N2;  // no second destination
  } else if (C2 == 0 || csplit % 4 || ldc2 % 4 || (C2 % 16) || splitk < 2 || workspace == 0) {
    throw std::invalid_argument("ccmpi gemm_tn: a column-split output needs split-K with a workspace, "
                                "csplit % 4 == 0 and a 16-B aligned second output");
  }
  if (N1 % 8 || N2 % 8 || lda % 8 || ldb % 8 || (A % 16) || (B % 16))
    throw std::invalid_argument("ccmpi gemm_tn: N1, N2, lda, ldb must be multiples of 8 and A/B 16-B aligned");
  if (splitk < 1) splitk = 1;
  // variant 1: 256x256 8-wave ping-pong TN kernel (gemm256.hip); partials of every
  // split go to workspace slices, then k_splitk_reduce
  if (variant == 1 && M % 128 == 0 && N1 >= 256 && N2 >= 256 && (C % 16) == 0 && ldc % 4 == 0 &&
      (splitk == 1 || (workspace != 0 && (workspace % 16) == 0))) {
    auto st = reinterpret_cast<hipStream_t>(stream);
    GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B),
               reinterpret_cast<void*>(splitk > 1 ? workspace : C), nullptr, N1, N2, M, lda, ldb,
               splitk > 1 ? N2 : ldc, alpha, (splitk == 1 && accumulate) ? 1 : 0, 0, 0, 0, splitk};
    launch_gemm_tn_256(g, st);
    CCMPI_HIP_CHECK(hipGetLastError());
    if (splitk > 1) {
      const size_t work = (size_t)N1 * (N2 / 4);
      const int grid = (int)std::min<size_t>((work + 255) / 256, 4096);
      hipLaunchKernelGGL(k_splitk_reduce, dim3(grid), dim3(256), 0, st, reinterpret_cast<const float*>(workspace), splitk,
                         reinterpret_cast<float*>(C), ldc, N1, N2, accumulate ? 1 : 0,
                         reinterpret_cast<float*>(C2), ldc2, csplit);
      CCMPI_HIP_CHECK(hipGetLastError());
    }
    return;
  }
  // split-K partials: a workspace of splitk fp32 slices summed by k_splitk_reduce
  // (coalesced stores + one streaming pass) instead of fp32 atomics on C
  const bool use_ws = splitk > 1 && workspace != 0 && N2 % 4 == 0 && ldc % 4 == 0 && (C % 16) == 0 &&
                      (workspace % 16) == 0;
  if (splitk > 1 && !accumulate && !use_ws)
    CCMPI_HIP_CHECK(hipMemset2DAsync(reinterpret_cast<void*>(C), (size_t)ldc * 4, 0, (size_t)N2 * 4, N1,
                                     reinterpret_cast<hipStream_t>(stream)));
  GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B),
             reinterpret_cast<void*>(use_ws ? workspace : C), nullptr, N1, N2, M, lda, ldb, use_ws ? N2 : ldc, alpha,
             accumulate ? 1 : 0, 0, 0, 0, splitk};
  const int nwg = ((N1 + BM - 1) / BM) * ((N2 + BN - 1) / BN) * splitk;
  const bool aligned = (C % 16) == 0 && ldc % 4 == 0 && N2 % 4 == 0;
  const int fast = use_ws ? 4 : !aligned ? 0 : splitk > 1 ? 1 : accumulate ? 3 : 2;
  auto st = reinterpret_cast<hipStream_t>(stream);
  // two K tiles in flight when each workgroup walks several of them (g_tn_pf: A/B knob)
  const int nk_split = ((M + BK - 1) / BK + splitk - 1) / splitk;
  // (PF = 2 addresses a split's rows with 32-bit buffer offsets)
  const bool fits = (size_t)nk_split * BK * std::max(lda, ldb) * 2 < (1ull << 31);
  const bool pf2 = fits && (g_tn_pf == 2 || (g_tn_pf == 0 && nk_split >= 4));
  if (pf2) {
    switch (fast) {
      case 4: hipLaunchKernelGGL((k_gemm_tn<4, 2>), dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
      case 1: hipLaunchKernelGGL((k_gemm_tn<1, 2>), dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
      case 2: hipLaunchKernelGGL((k_gemm_tn<2, 2>), dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
      case 3: hipLaunchKernelGGL((k_gemm_tn<3, 2>), dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
      default: hipLaunchKernelGGL((k_gemm_tn<0, 2>), dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
    }
    CCMPI_HIP_CHECK(hipGetLastError());
    if (fast == 4) {
      const size_t work = (size_t)N1 * (N2 / 4);
      const int grid = (int)std::min<size_t>((work + 255) / 256, 4096);
      hipLaunchKernelGGL(k_splitk_reduce, dim3(grid), dim3(256), 0, st, reinterpret_cast<const float*>(workspace), splitk,
                         reinterpret_cast<float*>(C), ldc, N1, N2, accumulate ? 1 : 0,
                         reinterpret_cast<float*>(C2), ldc2, csplit);
      CCMPI_HIP_CHECK(hipGetLastError());
    }
    return;
  }
  switch (fast) {
    case 4: {
      hipLaunchKernelGGL(k_gemm_tn<4>, dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major);
      CCMPI_HIP_CHECK(hipGetLastError());
      const size_t work = (size_t)N1 * (N2 / 4);
      const int grid = (int)std::min<size_t>((work + 255) / 256, 4096);
      hipLaunchKernelGGL(k_splitk_reduce, dim3(grid), dim3(256), 0, st, reinterpret_cast<const float*>(workspace), splitk,
                         reinterpret_cast<float*>(C), ldc, N1, N2, accumulate ? 1 : 0,
                         reinterpret_cast<float*>(C2), ldc2, csplit);
      break;
    }
    case 1: hipLaunchKernelGGL(k_gemm_tn<1>, dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
    case 2: hipLaunchKernelGGL(k_gemm_tn<2>, dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
    case 3: hipLaunchKernelGGL(k_gemm_tn<3>, dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
    default: hipLaunchKernelGGL(k_gemm_tn<0>, dim3(nwg), dim3(NT), 0, st, g, g_tn_split_major); break;
  }
  CCMPI_HIP_CHECK(hipGetLastError());
}

void transpose16(uint64_t src, uint64_t dst, int R, int C, int lds, int ldd, uint64_t stream) {
  if (R <= 0 || C <= 0) return;
  if (R % 8 == 0 && C % 8 == 0 && lds % 8 == 0 && ldd % 8 == 0 && src % 16 == 0 && dst % 16 == 0) {
    static const bool reg = std::getenv("CCMPI_TRANSPOSE") && std::string(std::getenv("CCMPI_TRANSPOSE")) == "reg";
    if (!reg) {  // the LDS tile by default; CCMPI_TRANSPOSE=reg picks the register transpose (A/B)
      dim3 grid((C + 63) / 64, (R + 63) / 64);
      hipLaunchKernelGGL(k_transpose16_l, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                         reinterpret_cast<const uint16_t*>(src), reinterpret_cast<uint16_t*>(dst), R, C, lds, ldd);
      CCMPI_HIP_CHECK(hipGetLastError());
      return;
    }
    dim3 grid((C + 63) / 64, (R + 511) / 512);
    hipLaunchKernelGGL(k_transpose16_v, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const uint16_t*>(src), reinterpret_cast<uint16_t*>(dst), R, C, lds, ldd);
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(k_transpose16, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const uint16_t*>(src), reinterpret_cast<uint16_t*>(dst), R, C, lds, ldd);
  CCMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void register_gemm_ops(pybind11::module_& m) {
  m.def("gemm_nt", &gemm_nt, "C = act(alpha*A.B^T + bias) (+C); A[M,K], B[N,K] bf16",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("bias"), pybind11::arg("M"),
        pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("lda"), pybind11::arg("ldb"), pybind11::arg("ldc"),
        pybind11::arg("alpha"), pybind11::arg("accumulate"), pybind11::arg("bias_kind"), pybind11::arg("act"),
        pybind11::arg("out_bf16"), pybind11::arg("splitk"), pybind11::arg("stream"),
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("gemm_ring", &gemm_ring,
        "LDS-ring GEMM, C (+)= alpha*op(A).op(B)^T with K-major (ta/tb=1) or K-contiguous operands; false = n/a",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("M"), pybind11::arg("N"),
        pybind11::arg("K"), pybind11::arg("lda"), pybind11::arg("ldb"), pybind11::arg("ldc"), pybind11::arg("ta"),
        pybind11::arg("tb"), pybind11::arg("alpha"), pybind11::arg("accumulate"), pybind11::arg("out_bf16"),
        pybind11::arg("stream"), pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("gemm_tn", &gemm_tn, "C[N1,N2] (+)= alpha*A[M,N1]^T.B[M,N2] (fp32 out; split-K via workspace or atomics)",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("M"), pybind11::arg("N1"),
        pybind11::arg("N2"), pybind11::arg("lda"), pybind11::arg("ldb"), pybind11::arg("ldc"), pybind11::arg("alpha"),
        pybind11::arg("accumulate"), pybind11::arg("splitk"), pybind11::arg("stream"), pybind11::arg("workspace") = 0,
        pybind11::arg("variant") = 0, pybind11::arg("C2") = 0, pybind11::arg("ldc2") = 0, pybind11::arg("csplit") = 0,
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("gemm_set_glds", [](bool on) { g_use_glds = on; }, "select LDS-DMA (True) or register staging");
  m.def("gemm_tn_set_prefetch", [](int pf) { g_tn_pf = pf; },
        "128x128 TN kernel: K tiles in flight (0 auto, 1, 2)", pybind11::arg("pf"));
  m.def("gemm_set_direct_epilogue", [](bool on) { g_direct_epi = on; },
        "128x128 LDS-DMA kernel: LDS-free epilogue (True) or LDS-staged rows");
  m.def("gemm_set_kernel", [](int k) { g_kernel = k; },
        "gemm_nt tile choice: 0 auto, 1 128x128, 2 256x256, 3 256x128, 4 256x192, 5 256x256 four-wave");
  m.def("gemm_set_w4_sched", [](int v) { g_w4_sched = v; },
        "four-wave kernel variant (benchmarks): bit 0 persistent grid, bit 1 MFMA-first group order");
  m.def("gemm_set_w4_debug", [](uint64_t p) { g_w4_dbg = reinterpret_cast<unsigned long long*>(p); },
        "four-wave ring STAMP diagnostic: device buffer of 4 uint64 per wave (benchmarks only)");
  m.def("gemm_set_ring_min", [](long long v) { g_ring_min_macs = v; },
        "gemm_nt auto: LDS-ring kernel from this many multiply-adds up (0 = never)");
  m.def("gemm_ring_launches", [] { return g_ring_launches; }, "LDS-ring GEMM launches so far (this process)");
  m.def("gemm_set_pair_nobar", [](int v) { g_pair_nobar = v; }, "diagnostic: pair ring without its barrier (wrong results)");
  m.def("gemm_set_pair_ta", [](int v) { g_pair_ta = v; }, "K-major A alone on the pair-slot ring (1) or the 4-slot ring (0)");
  m.def("gemm_set_ring_sched", [](int v) { g_ring_sched = v; },
        "auto-dispatched LDS-ring kernel variant: bit 3 ring, bit 14 pair slots (default), bit 0 persistent, bit 15 long K too; diagnostics: bits 5-6 / 13 ablations, bit 9 stamps");
  m.def("gemm_set_w4_group_m", [](int v) { g_w4_group_m = v > 0 ? v : 8; }, "four-wave kernel group-M rows");
  m.def("gemm_set_ablation", [](int e) {
    g_pp_exp = e;
    CCMPI_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pp_exp_dev), &e, sizeof(int)));
  }, "GEMM ablation bits (benchmarks only): 1/2/4 ping-pong kernel, 8 = skip the 128x128 epilogue");
  m.def("embed_patches", &embed_patches, "h = patches(x) . W^T (bf16), patch rows generated in-kernel and stored to xp",
        pybind11::arg("x"), pybind11::arg("W"), pybind11::arg("C"), pybind11::arg("B"), pybind11::arg("img"),
        pybind11::arg("p"), pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("ldw"), pybind11::arg("ldc"),
        pybind11::arg("xp"), pybind11::arg("ld_xp"), pybind11::arg("stream"),
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("gemm_set_smallk_nt", [](bool on) { g_sk_nt = on; }, "small-K kernel: non-temporal bf16 output stores");
  m.def("gemm_set_smallk", [](int bn, int grid) { g_sk_bn = bn; g_sk_grid = grid; },
        "small-K kernel: N slice (128 / 256, 0 = off) and grid cap (tuning)");
  m.def("transpose16", &transpose16, "dst[C,R] = src[R,C]^T for 16-bit elements",
        pybind11::call_guard<pybind11::gil_scoped_release>());
}

}  // namespace dev
}  // namespace ccmpi
