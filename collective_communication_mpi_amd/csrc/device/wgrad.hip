// Weight gradients of the harness's embedding -> QKV chain from the one
// token-length contraction A = dQKV^T . Xp (fp32 [R][kp], R = 3*hd rows of this
// TP rank, kp = 72 patch columns), in ONE launch:
//
//   Gq[R][d]  += A . We^T      (dW_qkv; h = Xp . We^T, so dQKV^T . h = A . We^T)
//   Ge[d][kp] += Wq^T . A      (dW_emb, or this TP rank's partial of it)
//   Z[R][kp]   = 0             (next step's A buffer: the split-K GEMM that forms A
//                               accumulates with atomics into a zeroed buffer, so
//                               no memset launch per step)
//
// Both products are tiny (85 and 42 MFLOP fp32) and latency-bound; two library
// sgemm launches took 6.7 + 9.0 us, plus a 5 us memset for A.
//
//   * Gq: 64 x 64 output tiles (144 workgroups at R = d = 768).  Both operand
//     tiles are staged K-major in LDS ([k][64 + 4] fp32), so a thread's 4 rows /
//     4 columns at one k are two 16-B LDS reads feeding 16 FMAs.
//   * Ge: 64-column tiles of d x 96-row splits of the R reduction (96 workgroups
//     at R = d = 768), operand slabs staged in LDS; the splits meet through fp32
//     atomic adds.
//   Every global operand load of a workgroup is issued before the first use (the
//   kernel is latency-bound: one serial load per loop trip cost 85 us).
#include <pybind11/pybind11.h>

#include "common.hpp"
#include "ops.hpp"

namespace ccmpi {
namespace dev {

namespace {

constexpr int kT = 64;          // Gq tile edge, Ge tile height (d columns)
constexpr int kLdT = kT + 4;    // LDS row stride (floats) of the K-major Gq tiles
constexpr int kMaxKp = 96;      // patch columns (kp % 4 == 0)
constexpr int kGeRows = 96;     // Ge: rows of the R reduction per workgroup
constexpr int kNT = 256;

struct WgradArgs {
  const float* A;
  int ld_a;
  const float* We;
  int ld_we;
  const float* Wq;
  int ld_wq;
  float* Gq;
  int ld_gq;
  float* Ge;
  int ld_ge;
  float* Z;
  int ld_z;
  int R, d, kp;
  int gq_blocks;   // workgroups [0, gq_blocks) do Gq tiles, the rest Ge partials
  int splits;      // Ge: R-splits per d tile
  int ge_mfma;     // Ge tiles on the matrix cores (ge_tile_mfma) instead of atomic R-splits
};

// Gq[r0.., c0..] += sum_k A[r][k] We[c][k] for a 64 x 64 tile.  Operand tiles are
// fetched with every float4 load in flight, then stored K-major to LDS so one
// thread's 4 rows / 4 columns at a k are two 16-B LDS reads for 16 FMAs.
__device__ void gq_tile(const WgradArgs& a, int blk, float* smem) {
  float* At = smem;                  // [kp][kLdT]: At[k][r] = A[r0 + r][k]
  float* Wt = smem + kMaxKp * kLdT;  // [kp][kLdT]: Wt[k][c] = We[c0 + c][k]
  const int tiles_c = (a.d + kT - 1) / kT;
  const int r0 = (blk / tiles_c) * kT, c0 = (blk % tiles_c) * kT;
  const int t = threadIdx.x, nv = a.kp / 4;
  const int tx = t & 15, ty = t >> 4;  // rows 4*ty.., columns 4*tx..
  // the tile's old Gq values are fetched with the operands (the read-modify-write at the
  // end would otherwise wait out a second memory round trip)
  float4 old[4];
  bool vec[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + 4 * ty + i;
    const float* g = a.Gq + (size_t)r * a.ld_gq + c0 + 4 * tx;
    vec[i] = r < a.R && c0 + 4 * tx + 3 < a.d && ((reinterpret_cast<uintptr_t>(g) & 15) == 0);
    old[i] = vec[i] ? *reinterpret_cast<const float4*>(g) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  constexpr int kPer = kT * (kMaxKp / 4) / kNT;  // float4 per thread per operand at kp = 96
  float4 ra[kPer], rw[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int idx = t + u * kNT, r = idx / nv, q = idx % nv;
    const bool ok = idx < kT * nv;
    ra[u] = (ok && r0 + r < a.R) ? *reinterpret_cast<const float4*>(a.A + (size_t)(r0 + r) * a.ld_a + 4 * q)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    rw[u] = (ok && c0 + r < a.d) ? *reinterpret_cast<const float4*>(a.We + (size_t)(c0 + r) * a.ld_we + 4 * q)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int idx = t + u * kNT, r = idx / nv, q = idx % nv;
    if (idx < kT * nv) {
      float* pa = At + 4 * q * kLdT + r;
      float* pw = Wt + 4 * q * kLdT + r;
      pa[0] = ra[u].x; pa[kLdT] = ra[u].y; pa[2 * kLdT] = ra[u].z; pa[3 * kLdT] = ra[u].w;
      pw[0] = rw[u].x; pw[kLdT] = rw[u].y; pw[2 * kLdT] = rw[u].z; pw[3 * kLdT] = rw[u].w;
    }
  }
  __syncthreads();
  float acc[4][4] = {};
  // unrolled so the LDS reads of several k are in flight (one k per trip waited out
  // the LDS latency every 16 FMAs)
#pragma unroll 8
  for (int k = 0; k < a.kp; ++k) {
    const float4 av = *reinterpret_cast<const float4*>(At + k * kLdT + 4 * ty);
    const float4 wv = *reinterpret_cast<const float4*>(Wt + k * kLdT + 4 * tx);
    const float ar[4] = {av.x, av.y, av.z, av.w}, wr[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(ar[i], wr[j], acc[i][j]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + 4 * ty + i;
    if (r >= a.R) continue;
    float* g = a.Gq + (size_t)r * a.ld_gq + c0 + 4 * tx;
    if (vec[i]) {
      float4 o = old[i];
      o.x += acc[i][0]; o.y += acc[i][1]; o.z += acc[i][2]; o.w += acc[i][3];
      *reinterpret_cast<float4*>(g) = o;
    } else {
      for (int j = 0; j < 4; ++j)
        if (c0 + 4 * tx + j < a.d) g[j] += acc[i][j];
    }
  }
}

// Ge partial of one (d tile, R split): P[i][j] = sum_{r in split} Wq[r][i0 + i] A[r][j]
// for 64 d columns x kp, both operand slabs staged row-major in LDS (all loads in
// flight); thread (i4, jg) owns d columns 4*i4.. and patch columns jg + 16m.
__device__ void ge_tile(const WgradArgs& a, int blk, float* smem) {
  constexpr int kLdW = kT + 4, kLdA = kMaxKp + 4;
  float* Ws = smem;                   // [kGeRows][kLdW]
  float* As = smem + kGeRows * kLdW;  // [kGeRows][kLdA]
  const int itile = blk / a.splits, split = blk % a.splits;
  const int i0 = itile * kT, rlo = split * kGeRows, rows = max(0, min(kGeRows, a.R - rlo));
  const int t = threadIdx.x, nv = a.kp / 4;
  constexpr int kPerW = kGeRows * (kT / 4) / kNT, kPerA = (kGeRows * (kMaxKp / 4) + kNT - 1) / kNT;
  float4 rw[kPerW], ra[kPerA];
#pragma unroll
  for (int u = 0; u < kPerW; ++u) {
    const int idx = t + u * kNT, r = idx / (kT / 4), q = idx % (kT / 4);
    rw[u] = (r < rows && i0 + 4 * q + 3 < a.d)
                ? *reinterpret_cast<const float4*>(a.Wq + (size_t)(rlo + r) * a.ld_wq + i0 + 4 * q)
                : make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < rows && i0 + 4 * q < a.d && i0 + 4 * q + 3 >= a.d) {  // ragged d edge
      const float* w = a.Wq + (size_t)(rlo + r) * a.ld_wq + i0 + 4 * q;
      rw[u].x = w[0];
      if (i0 + 4 * q + 1 < a.d) rw[u].y = w[1];
      if (i0 + 4 * q + 2 < a.d) rw[u].z = w[2];
    }
  }
#pragma unroll
  for (int u = 0; u < kPerA; ++u) {
    const int idx = t + u * kNT, r = idx / nv, q = idx % nv;
    ra[u] = (idx < kGeRows * nv && r < rows)
                ? *reinterpret_cast<const float4*>(a.A + (size_t)(rlo + r) * a.ld_a + 4 * q)
                : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < kPerW; ++u) {
    const int idx = t + u * kNT, r = idx / (kT / 4), q = idx % (kT / 4);
    *reinterpret_cast<float4*>(Ws + r * kLdW + 4 * q) = rw[u];
  }
#pragma unroll
  for (int u = 0; u < kPerA; ++u) {
    const int idx = t + u * kNT, r = idx / nv, q = idx % nv;
    if (idx < kGeRows * nv) *reinterpret_cast<float4*>(As + r * kLdA + 4 * q) = ra[u];
  }
  __syncthreads();
  const int i4 = t & 15, jg = t >> 4;
  float acc[6][4] = {};
#pragma unroll 8
  for (int r = 0; r < rows; ++r) {
    const float4 w4 = *reinterpret_cast<const float4*>(Ws + r * kLdW + 4 * i4);
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      const float x = As[r * kLdA + jg + 16 * m];  // columns >= kp hold junk, never stored
      acc[m][0] = fmaf(w4.x, x, acc[m][0]);
      acc[m][1] = fmaf(w4.y, x, acc[m][1]);
      acc[m][2] = fmaf(w4.z, x, acc[m][2]);
      acc[m][3] = fmaf(w4.w, x, acc[m][3]);
    }
  }
  // fp32 atomic adds into Ge (hardware global_atomic_add_f32, no return): the R
  // splits meet in memory.  A ticket-and-last-workgroup reduction (fixed order)
  // cost ~20 us here -- agent-coherent hand-off plus a serial partial read -- and
  // A itself is already a split-K atomic sum, so order-exact sums bought nothing.
  // The tile goes through LDS first so each wave-instruction adds 64 consecutive
  // floats of a row: straight from the accumulator layout an instruction touched 16
  // rows x 16 B, and the adds ran ~8x below the atomic rate (8 of the kernel's 15 us).
  constexpr int kLdP = kMaxKp + 1;
  __syncthreads();  // every wave is done with the operand slabs
  float* tile = smem;  // [kT][kLdP]
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const int j = jg + 16 * m;
    if (j < a.kp)
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[(4 * i4 + e) * kLdP + j] = acc[m][e];
  }
  __syncthreads();
  for (int idx = t; idx < kT * a.kp; idx += kNT) {
    const int i = idx / a.kp, j = idx % a.kp;
    if (i0 + i < a.d) unsafeAtomicAdd(a.Ge + (size_t)(i0 + i) * a.ld_ge + j, tile[i * kLdP + j]);
  }
}

// Ge on the fp32 matrix cores (R <= 768): one 16 x 16 tile of Ge = Wq^T A per workgroup over
// ALL R rows, so no atomics -- the tile is read, added to and written once.  The 4 waves take
// R / 4 rows each: MFMA m of wave w covers rows 4 (w G + m) .. +3 (G = groups per wave), lane
// (c, g) supplying Wq[row g][i0 + c] and A[row g][j0 + c] (both 64-B coalesced), every load
// issued before the first MFMA; the 4 partial tiles are summed in wave order in LDS.  (The
// 8 R-splits x 64-column atomic tiles of ge_tile cost 5 us of the kernel's 12.)
constexpr int kGeMaxG = 48;  // 4-row groups per wave: R <= 4 * 4 * 48
// Ge variant (wgrad_set_ge_mfma / CCMPI_WGRAD_GE=atomic for the R-split atomic tiles)
bool g_ge_mfma = std::getenv("CCMPI_WGRAD_GE") == nullptr || std::string(std::getenv("CCMPI_WGRAD_GE")) != "atomic";

__device__ void ge_tile_mfma(const WgradArgs& a, int blk, float* smem) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int tiles_j = (a.kp + 15) / 16;
  const int i0 = (blk / tiles_j) * 16, j0 = (blk % tiles_j) * 16;
  const int ngroups = (a.R + 3) / 4, G = (ngroups + 3) / 4;
  const bool iok = i0 + c < a.d, jok = j0 + c < a.kp;
  // the tile's old values, fetched with the operands (lane: row 4g + r, column c)
  float old[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    old[r] = (wave == 0 && i < a.d && jok) ? a.Ge[(size_t)i * a.ld_ge + j0 + c] : 0.f;
  }
  float wv[kGeMaxG], av[kGeMaxG];
#pragma unroll
  for (int m = 0; m < kGeMaxG; ++m) {
    const int row = 4 * (wave * G + m) + g;
    const bool ok = m < G && row < a.R;
    wv[m] = (ok && iok) ? a.Wq[(size_t)row * a.ld_wq + i0 + c] : 0.f;
    av[m] = (ok && jok) ? a.A[(size_t)row * a.ld_a + j0 + c] : 0.f;
  }
  f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < kGeMaxG; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[m], av[m], acc, 0, 0, 0);
  float* part = smem;  // [4][16][17]
#pragma unroll
  for (int r = 0; r < 4; ++r) part[(wave * 16 + 4 * g + r) * 17 + c] = acc[r];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * g + r;
      const float v = part[i * 17 + c] + part[(16 + i) * 17 + c] + part[(32 + i) * 17 + c] + part[(48 + i) * 17 + c];
      if (i0 + i < a.d && jok) a.Ge[(size_t)(i0 + i) * a.ld_ge + j0 + c] = old[r] + v;
    }
  }
}

constexpr size_t kSmemFloats = 2 * kMaxKp * kLdT > kGeRows * (kT + 4 + kMaxKp + 4)
                                   ? 2 * kMaxKp * kLdT : kGeRows * (kT + 4 + kMaxKp + 4);

__global__ void __launch_bounds__(kNT) k_emb_qkv_wgrad(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[kSmemFloats];
  const int blk = blockIdx.x;
  // (dW_qkv on the matrix cores as 2 x 2 MFMA tiles per wave measured 6.8 us alone but 9.4 us
  // beside the dW_emb tiles, against 7.2 / 8.2 for these FMA tiles: not kept)
  if (blk < a.gq_blocks) gq_tile(a, blk, smem);
  else if (a.Ge && a.ge_mfma) ge_tile_mfma(a, blk - a.gq_blocks, smem);
  else if (a.Ge) ge_tile(a, blk - a.gq_blocks, smem);
  if (a.Z) {  // zero the next A buffer, spread over every workgroup
    const size_t n = (size_t)a.R * a.kp;
    for (size_t e = (size_t)blk * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
      a.Z[(e / a.kp) * a.ld_z + e % a.kp] = 0.f;
  }
}

void emb_qkv_wgrad(uint64_t A, int ld_a, uint64_t We, int ld_we, uint64_t Wq, int ld_wq, uint64_t Gq, int ld_gq,
                   uint64_t Ge, int ld_ge, uint64_t Z, int ld_z, int R, int d, int kp, uint64_t stream) {
  if (R <= 0 || d <= 0 || kp <= 0) return;
  if (kp > kMaxKp || kp % 4 || ld_a % 4 || ld_we % 4 || ld_wq % 4 || (A % 16) || (We % 16) || (Wq % 16))
    throw std::invalid_argument("emb_qkv_wgrad: kp <= 96, kp and row strides % 4 == 0, 16-B aligned operands");
  if (!A || !We || !Gq || (Z && Z == A)) throw std::invalid_argument("emb_qkv_wgrad: A, We, Gq required; Z must differ from A");
  if (Ge && !Wq) throw std::invalid_argument("emb_qkv_wgrad: Ge needs Wq");
  const int splits = (R + kGeRows - 1) / kGeRows, dtiles = (d + kT - 1) / kT;
  WgradArgs a{reinterpret_cast<const float*>(A), ld_a, reinterpret_cast<const float*>(We), ld_we,
              reinterpret_cast<const float*>(Wq), ld_wq, reinterpret_cast<float*>(Gq), ld_gq,
              reinterpret_cast<float*>(Ge), ld_ge, reinterpret_cast<float*>(Z), ld_z, R, d, kp, 0, splits};
  a.gq_blocks = ((R + kT - 1) / kT) * dtiles;
  a.ge_mfma = (g_ge_mfma && R <= 4 * 4 * kGeMaxG) ? 1 : 0;
  const int ge_blocks = !Ge ? 0 : a.ge_mfma ? ((d + 15) / 16) * ((kp + 15) / 16) : dtiles * splits;
  hipLaunchKernelGGL(k_emb_qkv_wgrad, dim3(a.gq_blocks + ge_blocks), dim3(kNT), 0, (hipStream_t)stream, a);
  CCMPI_HIP_CHECK(hipGetLastError());
}

// Forward weight fold of the same chain: h = Xp . We^T feeds only qkv = h . Wq^T + b
// (no nonlinearity between), so qkv = Xp . Weff^T + b with
//
//   Weff[R][kp] = Wq[R][d] . We[d][kp]   (fp32 accumulate, bf16 out)
//
// and the forward runs one K = kp GEMM instead of K = kp plus K = d (the d = 768
// QKV GEMM was 54 of the 184 us train step).  Same role as the weight-side
// contractions above: a tiny, latency-bound fp32 product (42 MFLOP at 768 x 72).
//   * one 512-thread workgroup per kFoldRows (3) rows of Weff; their Wq rows are staged
//     in LDS;
//   * thread (slice, cg): patch columns 4*cg.. (one float4 of a We row per k),
//     k = slice, slice + ns, ... (interleaved, so the slices' LDS reads of one Wq
//     row hit distinct banks; the column groups of one slice broadcast);
//   * every global load of a thread -- its Wq chunks and its kFoldBatch We rows --
//     is issued before the first use: at d = 768 that is ONE memory round trip
//     (one load per loop trip: 19 us; 16 rows per trip: 13.7 us);
//   * the ns slice partials meet in LDS in two fixed-order halves (deterministic).
constexpr int kFoldNT = 512;
constexpr int kFoldRows = 3;  // 256 workgroups at R = 768: every CU (8 rows: 96 CUs, 10.2 us)
constexpr int kFoldBatch = 28;  // d = 768: 28 slices x 28 rows, one trip (32 spilled VGPRs)
constexpr int kFoldMaxD = 1024;
constexpr int kFoldWqPer = (kFoldRows * kFoldMaxD / 4 + kFoldNT - 1) / kFoldNT;  // float4 of Wq per thread

__global__ void __launch_bounds__(kFoldNT) k_fold_emb_qkv(const float* __restrict__ Wq, int ld_wq,
                                                          const float* __restrict__ We, int ld_we,
                                                          uint16_t* __restrict__ Weff, int ld_eff, int R, int d, int kp,
                                                          const float* __restrict__ bias, int bias_col) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int t = threadIdx.x, r0 = blockIdx.x * kFoldRows, nv = d / 4;
  const int ng = kp / 4, ns = kFoldNT / ng, slice = t / ng, cg = t % ng;
  const bool act = slice < ns;
  float4 wq[kFoldWqPer];
#pragma unroll
  for (int u = 0; u < kFoldWqPer; ++u) {
    const int idx = t + u * kFoldNT, r = idx / nv, q = idx % nv;
    wq[u] = (idx < kFoldRows * nv && r0 + r < R) ? *reinterpret_cast<const float4*>(Wq + (size_t)(r0 + r) * ld_wq + 4 * q)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 w[kFoldBatch];
  auto fetch = [&](int kb) {
#pragma unroll
    for (int u = 0; u < kFoldBatch; ++u) {
      const int k = kb + u * ns;
      w[u] = (act && k < d) ? *reinterpret_cast<const float4*>(We + (size_t)k * ld_we + 4 * cg) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  int kb = slice;
  fetch(kb);
#pragma unroll
  for (int u = 0; u < kFoldWqPer; ++u) {
    const int idx = t + u * kFoldNT;
    if (idx < kFoldRows * nv) *reinterpret_cast<float4*>(fsm + 4 * idx) = wq[u];  // row r at fsm + r * d
  }
  __syncthreads();
  float acc[kFoldRows][4] = {};
  while (true) {
#pragma unroll
    for (int u = 0; u < kFoldBatch; ++u) {
      const int k = min(kb + u * ns, d - 1);  // past d: w[u] == 0, any in-range row
#pragma unroll
      for (int r = 0; r < kFoldRows; ++r) {
        const float x = fsm[r * d + k];
        acc[r][0] = fmaf(x, w[u].x, acc[r][0]);
        acc[r][1] = fmaf(x, w[u].y, acc[r][1]);
        acc[r][2] = fmaf(x, w[u].z, acc[r][2]);
        acc[r][3] = fmaf(x, w[u].w, acc[r][3]);
      }
    }
    kb += kFoldBatch * ns;
    if (kb >= d) break;
    fetch(kb);
  }
  // partials: slices [half, ns) write position slice - half, then slices [0, half) add
  // theirs in place; the half positions are summed in order
  const int half = (ns + 1) / 2;
  __syncthreads();  // every slice is done with the Wq rows: reuse the LDS
  auto slot = [&](int pos, int r) { return reinterpret_cast<float4*>(fsm + (pos * kFoldRows + r) * kp + 4 * cg); };
  if (act && slice >= half)
#pragma unroll
    for (int r = 0; r < kFoldRows; ++r) *slot(slice - half, r) = make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
  __syncthreads();
  if (slice < half) {
    const bool pair = slice + half < ns;
#pragma unroll
    for (int r = 0; r < kFoldRows; ++r) {
      float4 v = make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
      if (pair) {
        const float4 o = *slot(slice, r);
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      *slot(slice, r) = v;
    }
  }
  __syncthreads();
  for (int idx = t; idx < kFoldRows * kp; idx += kFoldNT) {
    const int r = idx / kp, c = idx % kp;
    if (r0 + r >= R) continue;
    float s = 0.f;
    for (int p = 0; p < half; ++p) s += fsm[(p * kFoldRows + r) * kp + c];
    if (bias && c == bias_col) s += bias[r0 + r];  // Xp's constant-1 column carries the QKV bias
    Weff[(size_t)(r0 + r) * ld_eff + c] = static_cast<uint16_t>(f32_to_bf16_bits(s));
  }
}

// The same fold on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32
// accumulate): one 1024-thread workgroup per 16 x 16 tile of Weff (grid R/16 x kp/16 = 240
// workgroups at 768 x 72), its 16 waves splitting d.  A wave issues ALL its loads first --
// per 16-deep k chunk j one float4 of its Wq row (k = 16 j + 4 g .. +3: the MFMA's k slot g
// takes k = 16 j + 4 g + i at step i, the same permutation on both operands) and 4 We values
// -- so the whole product is one memory round trip, then 4 MFMAs per chunk.  The 16 wave
// partials meet in LDS in wave order (deterministic), + the bias column, bf16 out.  (A first
// version with one workgroup per 16 rows x all columns -- 48 workgroups, a load round trip
// per chunk -- took 17.9 us against the FMA kernel's 7.4 us.)
constexpr int kFmWaves = 16;  // (8: 4.9 us at 768 x 72 x 768, one 6-chunk load chain per wave)
constexpr int kFmMaxJ = 4;   // chunks per wave: d <= 16 * 4 * 16 = 1024

__global__ void __launch_bounds__(kFmWaves * 64) k_fold_mfma(const float* __restrict__ Wq, int ld_wq,
                                                            const float* __restrict__ We, int ld_we,
                                                            uint16_t* __restrict__ Weff, int ld_eff, int R, int d,
                                                            int kp, const float* __restrict__ bias, int bias_col) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float part[kFmWaves][16][16 + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * 16, c0 = blockIdx.y * 16, col = c0 + c;
  const int nj = (d + 15) / 16, per = (nj + kFmWaves - 1) / kFmWaves;
  const int j0 = wave * per;
  const bool rok = r0 + c < R, cok = col < kp;
  const float* arow = Wq + (size_t)(rok ? r0 + c : 0) * ld_wq;
  float4 a4[kFmMaxJ];
  float b[kFmMaxJ][4];
#pragma unroll
  for (int u = 0; u < kFmMaxJ; ++u) {
    const int k = 16 * (j0 + u) + 4 * g;  // d % 4 == 0: the float4 is all in range or all out
    const bool kok = u < per && k < d;
    a4[u] = (rok && kok) ? *reinterpret_cast<const float4*>(arow + k) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) b[u][i] = (cok && kok) ? We[(size_t)(k + i) * ld_we + col] : 0.f;
  }
  f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < kFmMaxJ; ++u) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].x, b[u][0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].y, b[u][1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].z, b[u][2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].w, b[u][3], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wave][4 * g + r][c] = acc[r];  // [row 4g + r][col c]
  __syncthreads();
  if (threadIdx.x < 256) {
    const int r = threadIdx.x >> 4, cc = threadIdx.x & 15;
    if (r0 + r < R && c0 + cc < kp) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < kFmWaves; ++w) sum += part[w][r][cc];
      if (bias && c0 + cc == bias_col) sum += bias[r0 + r];  // Xp's constant-1 column carries the QKV bias
      Weff[(size_t)(r0 + r) * ld_eff + c0 + cc] = static_cast<uint16_t>(f32_to_bf16_bits(sum));
    }
  }
}

int g_fold_variant = -1;  // -1: CCMPI_FOLD (default "mfma"), 0: FMA kernel, 1: MFMA kernel

size_t fold_lds_bytes(int d, int kp) {
  const int half = (kFoldNT / (kp / 4) + 1) / 2;
  return sizeof(float) * std::max<size_t>((size_t)kFoldRows * d, (size_t)half * kFoldRows * kp);
}

void fold_emb_qkv(uint64_t Wq, int ld_wq, uint64_t We, int ld_we, uint64_t Weff, int ld_eff, int R, int d, int kp,
                  uint64_t stream, uint64_t bias, int bias_col) {
  if (bias && (bias_col < 0 || bias_col >= kp)) throw std::invalid_argument("fold_emb_qkv: bias_col outside [0, kp)");
  if (R <= 0 || d <= 0 || kp <= 0) return;
  if (kp > kMaxKp || kp % 4 || d % 4 || d > kFoldMaxD || ld_wq % 4 || ld_we % 4 || (Wq % 16) || (We % 16) || !Weff)
    throw std::invalid_argument("fold_emb_qkv: kp <= 96, d <= 1024, kp / d / fp32 row strides % 4 == 0, 16-B aligned fp32 operands");
  if (g_fold_variant < 0) {
    const char* e = std::getenv("CCMPI_FOLD");
    g_fold_variant = (e && std::string(e) == "fma") ? 0 : 1;
  }
  if (g_fold_variant == 1) {
    hipLaunchKernelGGL(k_fold_mfma, dim3((R + 15) / 16, (kp + 15) / 16), dim3(kFmWaves * 64), 0, (hipStream_t)stream,
                       reinterpret_cast<const float*>(Wq), ld_wq, reinterpret_cast<const float*>(We), ld_we,
                       reinterpret_cast<uint16_t*>(Weff), ld_eff, R, d, kp, reinterpret_cast<const float*>(bias), bias_col);
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  const size_t lds = fold_lds_bytes(d, kp);
  if (lds > 64 * 1024) throw std::invalid_argument("fold_emb_qkv: LDS staging exceeds 64 KiB");
  hipLaunchKernelGGL(k_fold_emb_qkv, dim3((R + kFoldRows - 1) / kFoldRows), dim3(kFoldNT), lds, (hipStream_t)stream,
                     reinterpret_cast<const float*>(Wq), ld_wq, reinterpret_cast<const float*>(We), ld_we,
                     reinterpret_cast<uint16_t*>(Weff), ld_eff, R, d, kp, reinterpret_cast<const float*>(bias), bias_col);
  CCMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

// The fused forward's weight fold when it has more tiles than that kernel has workgroups
// (attn_mfma.hip launch_qkv_fwd_mfma): the fp32-MFMA kernel -- bitwise the in-kernel fold,
// whatever CCMPI_FOLD selects for the standalone fold
void fold_emb_qkv_mfma(const float* Wq, int ld_wq, const float* We, int ld_we, uint16_t* Weff, int ld_eff, int R, int d,
                       int kp, hipStream_t stream) {
  hipLaunchKernelGGL(k_fold_mfma, dim3((R + 15) / 16, (kp + 15) / 16), dim3(kFmWaves * 64), 0, stream, Wq, ld_wq, We,
                     ld_we, Weff, ld_eff, R, d, kp, nullptr, -1);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void register_wgrad_ops(pybind11::module_& m) {
  m.def("fold_emb_qkv", &fold_emb_qkv,
        "Weff (bf16) = Wq . We (+ bias in column bias_col), fp32 accumulate, fixed summation order",
        pybind11::arg("Wq"), pybind11::arg("ld_wq"), pybind11::arg("We"), pybind11::arg("ld_we"), pybind11::arg("Weff"),
        pybind11::arg("ld_eff"), pybind11::arg("R"), pybind11::arg("d"), pybind11::arg("kp"), pybind11::arg("stream"),
        pybind11::arg("bias") = 0, pybind11::arg("bias_col") = -1, pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("wgrad_set_ge_mfma", [](bool on) { g_ge_mfma = on; },
        "emb_qkv_wgrad's dW_emb part: matrix-core tiles over all R rows (True) or R-split atomic tiles",
        pybind11::arg("on"));
  m.def("fold_set_variant", [](int v) { g_fold_variant = v; },
        "fold_emb_qkv kernel: 0 = fp32 FMA, 1 = fp32 MFMA, -1 = CCMPI_FOLD (default mfma)", pybind11::arg("v"));
  m.def("emb_qkv_wgrad", &emb_qkv_wgrad,
        "Gq += A . We^T (fixed order); Ge += Wq^T . A (fp32 atomics; Ge = 0: skipped); Z = 0 (Z = 0: skipped)",
        pybind11::arg("A"), pybind11::arg("ld_a"), pybind11::arg("We"), pybind11::arg("ld_we"), pybind11::arg("Wq"),
        pybind11::arg("ld_wq"), pybind11::arg("Gq"), pybind11::arg("ld_gq"), pybind11::arg("Ge"), pybind11::arg("ld_ge"),
        pybind11::arg("Z"), pybind11::arg("ld_z"), pybind11::arg("R"), pybind11::arg("d"), pybind11::arg("kp"),
        pybind11::arg("stream"), pybind11::call_guard<pybind11::gil_scoped_release>());
}

}  // namespace dev
}  // namespace ccmpi
