// Short-sequence attention on matrix cores (S <= 16 keys/queries per
// sequence, head_dim D in {32, 64, 128}): the MNIST harness's 16-patch
// attention, forward and backward.  One wave per (sequence, local head), four
// waves per workgroup, grid-strided over the (b, h) pairs.
//
// Everything stays in MFMA register layouts (16x16 tiles; g = lane >> 4,
// c = lane & 15; an accumulator holds element [4g + r][c] in register r):
//   * Q, K, V, dO, O rows are read straight from the fused QKV buffer with one
//     16-B load per lane per 32 columns: lane (c, g) holds row c, columns
//     32kk + 8g .. +7 -- the A/B operand layout of v_mfma_f32_16x16x32_bf16.
//   * S^T = K Q^T (2 MFMAs at D = 64) leaves column i = query on the lane and
//     the 16 keys j = 4g + r in registers, so the softmax over j is 4 register
//     ops plus two cross-lane-group shuffles, and the probabilities P[i][4g + r]
//     ARE the A operand of v_mfma_f32_16x16x16_bf16 for O = P V (no lane
//     movement).  The V operand (4 consecutive keys of one column per lane) is
//     read from a per-wave LDS copy of the tile.
//   * Backward recomputes both S and S^T (and dP, dP^T), so each of
//     dV = P^T dO, dK = scale dS^T Q and dQ = scale dS K contracts over an
//     accumulator's row index: the accumulator is the A operand, the other
//     factor comes from the per-wave LDS tile.  delta_i = rowsum(dO * O) is
//     computed as rowsum(P * dP) from registers, so O is not read -- and the
//     forward skips storing O when the caller passes o = null (pooled mode).
//   * Outputs are staged per wave through LDS and written as 16-B row
//     vectors.  The pooled forward output (mean over the S rows, for the
//     pooled row-parallel fc_o) and the QKV bias gradient (column sums of dQ,
//     dK, dV) are reduced in registers; bias sums are flushed with one atomic
//     per column per wave (and whenever a wave's head changes).
// The kernel is memory bound (a few KiB moved per ~10 MFMAs): its cost is the
// QKV read and the O / dQKV write.
//
// The harness forward runs the fused form instead (k_qkv_attn16_fwd, attn16_fwd_body with
// QKV = true): patchify + QKV projection + attention + per-token fc_o (+ token mean, or the TP
// push into the peers' inboxes) + optionally the next step's weight fold, one kernel.  Persistent
// 8-wave workgroups, one per CU; W_h staged once per workgroup by LDS-DMA and held in registers;
// each wave reads its X fragments straight from the images in LDS (LDS-DMA two blocks ahead); a
// fold-aware block schedule (fold owners take fewer pair blocks, or at small batches the fold gets
// workgroups of its own); and lean instantiations carrying only the paths they take -- the
// instruction cache, not the arithmetic, set the last 10 % (profiles/r6_attn/README.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "attn_common.hpp"
#include "common.hpp"

namespace ccmpi {
namespace dev {
// wgrad.hip: the standalone fp32-MFMA weight fold (a fold too large for the fused kernel's grid)
void fold_emb_qkv_mfma(const float* Wq, int ld_wq, const float* We, int ld_we, uint16_t* Weff, int ld_eff, int R, int d,
                       int kp, hipStream_t stream);
namespace attn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int WPB = 4;  // waves per workgroup

__device__ __forceinline__ s4 pack4(float a, float b, float c, float d) {
  const uint2 u{pk_bf16(a, b), pk_bf16(c, d)};
  return __builtin_bit_cast(s4, u);
}
__device__ __forceinline__ bf16x8 ld_row16(const uint16_t* p, bool ok) {
  const uint4 z = ok ? *reinterpret_cast<const uint4*>(p) : uint4{0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, z);
}
__device__ __forceinline__ f4 mma32(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mma16(s4 a, s4 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }

// B operand of the 16x16x16 MFMA from a row-major [16][LD] bf16 LDS tile:
// lane (c, g) takes rows 4g..4g+3 of column col.
template <int LD>
__device__ __forceinline__ s4 tile_b(const uint16_t* T, int g, int col) {
  s4 r;
  r[0] = (short)T[(4 * g + 0) * LD + col];
  r[1] = (short)T[(4 * g + 1) * LD + col];
  r[2] = (short)T[(4 * g + 2) * LD + col];
  r[3] = (short)T[(4 * g + 3) * LD + col];
  return r;
}

// lane (c, g) wrote rows of a [16][D] result as accumulators [4g + r][16nt + c]:
// stage them as bf16 and store rows < S as 16-B vectors.
template <int D, int LD>
__device__ __forceinline__ void store_tile(uint16_t* T, const f4 (&v)[D / 16], float mul, uint16_t* dst, int ld, int S,
                                           int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < D / 16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) T[(4 * g + r) * LD + 16 * nt + c] = (uint16_t)f32_to_bf16_bits(v[nt][r] * mul);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int t = 0; t < (16 * D / 8) / 64; ++t) {
    const int p = lane + 64 * t, row = p / (D / 8), col = (p % (D / 8)) * 8;
    if (row < S) *reinterpret_cast<uint4*>(dst + (size_t)row * ld + col) = *reinterpret_cast<const uint4*>(T + row * LD + col);
  }
  __builtin_amdgcn_wave_barrier();
}

// copy register rows (lane (c, g): row c, columns 32kk + 8g..) into an LDS tile
template <int D, int LD>
__device__ __forceinline__ void put_rows(uint16_t* T, const bf16x8 (&x)[D / 32], int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) *reinterpret_cast<bf16x8*>(T + c * LD + 32 * kk + 8 * g) = x[kk];
}

// Reductions across the 16-lane rows of a wave on gfx950's v_permlane16/32_swap (VALU, no LDS
// round trip like the ds_bpermute behind __shfl_xor): with both operands = v, the two results
// hold, on every lane, v and its partner's v (lane ^ 16, resp. lane ^ 32), so op(r0, r1) is
// the pair reduction -- the same operand order on both partners, bitwise equal to the
// shuffle form.
__device__ __forceinline__ float pair16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pair32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pair16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// DPP row rotation: lane l of each 16-lane row reads lane (l - N) mod 16 of the same row
template <int N>
__device__ __forceinline__ float row_ror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + N, 0xf, 0xf, false));
}

__device__ __forceinline__ s4 ld_s4(const uint16_t* p, bool ok) {
  const uint2 z = ok ? *reinterpret_cast<const uint2*>(p) : uint2{0, 0};
  return __builtin_bit_cast(s4, z);
}

// copy the rows < S of a per-wave [16][LD] bf16 tile to global memory as 16-B vectors
template <int D, int LD>
__device__ __forceinline__ void rows_out(const uint16_t* T, uint16_t* dst, int ld, int S, int lane) {
#pragma unroll
  for (int t = 0; t < (16 * D / 8) / 64; ++t) {
    const int p = lane + 64 * t, row = p / (D / 8), col = (p % (D / 8)) * 8;
    if (row < S) *reinterpret_cast<uint4*>(dst + (size_t)row * ld + col) = *reinterpret_cast<const uint4*>(T + row * LD + col);
  }
}

// The forward body.  QKV = false: q, k, v rows are read from the qkv buffer (k_attn16_fwd).
// QKV = true (k_qkv_attn16_fwd, the harness forward with fc_o_mode "token"): the wave forms
// its (sequence, head)'s q | k | v = X W_h^T + b itself on the MFMA from the sequence's patch
// rows X (B*S x kq bf16, kq <= 80: two 16x16x32 k-steps + one 16x16x16 tail).  With Hl | WPB
// a wave always serves head h = wave % Hl, so W_h's 3 D x kq operand fragments (120 VGPRs at
// D = 64) are loaded ONCE and stay in registers for the whole block loop (workgroups are
// persistent: one 8-wave workgroup per CU); each iteration reads only X (patch-row mode:
// prefetched one iteration ahead; image mode: from the images LDS-DMA'd two blocks ahead).
// q and k are rounded to bf16 (the values the unfused QKV GEMM would store)
// and turned into row fragments through the wave's O / V tiles, v lands in the V tile the PV
// product reads; qkv is written only when a backward needs it (qkv_out).  The QKV GEMM's
// launch, its 2 x B*S x 3 Hl D x 2 B of qkv write + read, and the old per-head W staging
// (one wave per sequence, two workgroup barriers per head: 38.9 us vs 23.1 + 17.0 us
// unfused) are gone.
constexpr int kFoldSlices = 16, kFoldMaxJ = 4;  // the weight fold's K slices (see fold_tail)

// One 16 x 16 fold tile in three steps, so the fused kernel can put the operand loads in flight
// with its own prologue loads and share its barriers: fold_issue (operands into registers: each
// wave's K slices), fold_mma (the slices' MFMA chains -> partial tiles in LDS), fold_reduce (the
// first 256 threads sum the 16 partials in slice order and store).
template <int NW>
struct FoldOps {
  static constexpr int SPW = kFoldSlices / NW;  // K slices per wave (4 waves: 4, 8 waves: 2)
  float4 a4[SPW][kFoldMaxJ];
  float b[SPW][kFoldMaxJ][4];
};

__device__ __forceinline__ int fold_tiles(const AttnArgs& a) {
  return ((a.fold_R + 15) / 16) * ((a.fold_kp + 15) / 16);
}

template <int NW>
__device__ __forceinline__ void fold_issue(const AttnArgs& a, int tile, FoldOps<NW>& f) {
  constexpr int SPW = FoldOps<NW>::SPW;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int R = a.fold_R, d = a.fold_d, kp = a.fold_kp, tiles_c = (kp + 15) / 16;
  const int nj = (d + 15) / 16, per = (nj + kFoldSlices - 1) / kFoldSlices;
  const int r0 = (tile / tiles_c) * 16, col = (tile % tiles_c) * 16 + c;
  const bool rok = r0 + c < R, cok = col < kp;
  const float* arow = a.fold_wq + (size_t)(rok ? r0 + c : 0) * a.ld_fold_wq;
#pragma unroll
  for (int s = 0; s < SPW; ++s) {
    const int j0 = (SPW * wave + s) * per;
#pragma unroll
    for (int u = 0; u < kFoldMaxJ; ++u) {
      const int k = 16 * (j0 + u) + 4 * g;
      const bool kok = u < per && k < d;
      f.a4[s][u] = (rok && kok) ? *reinterpret_cast<const float4*>(arow + k) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < 4; ++i) f.b[s][u][i] = (cok && kok) ? a.fold_we[(size_t)(k + i) * a.ld_fold_we + col] : 0.f;
    }
  }
}

template <int NW>
__device__ __forceinline__ void fold_mma(const FoldOps<NW>& f, float* part /* 16 * 16 * 17 floats */) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  constexpr int SPW = FoldOps<NW>::SPW;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int s = 0; s < SPW; ++s) {
    f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < kFoldMaxJ; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a4[s][u].x, f.b[s][u][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a4[s][u].y, f.b[s][u][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a4[s][u].z, f.b[s][u][2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a4[s][u].w, f.b[s][u][3], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) part[((SPW * wave + s) * 16 + 4 * g + r) * 17 + c] = acc[r];
  }
}

__device__ __forceinline__ void fold_reduce(const AttnArgs& a, int tile, const float* part) {
  const int tiles_c = (a.fold_kp + 15) / 16;
  const int r0 = (tile / tiles_c) * 16, c0 = (tile % tiles_c) * 16;
  const int r = threadIdx.x >> 4, cc = threadIdx.x & 15;  // the first 256 threads: one output each
  if (threadIdx.x < 256 && r0 + r < a.fold_R && c0 + cc < a.fold_kp) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < kFoldSlices; ++w) sum += part[(w * 16 + r) * 17 + cc];
    a.fold_out[(size_t)(r0 + r) * a.ld_fold_out + c0 + cc] = static_cast<uint16_t>(f32_to_bf16_bits(sum));
  }
}

// The weight fold W_eff = bf16(Wq . We) as the tail of the fused forward (AttnArgs fold_*): one
// 16 x 16 output tile per workgroup and trip, the K axis cut into 16 slices exactly as wgrad.hip's
// k_fold_mfma cuts it over its 16 waves, the 16 partial tiles summed in slice order in LDS:
// bitwise that kernel's output, without its launch.  Tiles from `first` in steps of the grid.
template <int NW>
__device__ __forceinline__ void fold_tail(const AttnArgs& a, float* part /* >= 16 * 16 * 17 floats of LDS */,
                                          int first = -1) {
  // (tiles from the last workgroup down measured 0.0237-0.0239 vs 0.0232-0.0233 ms per forward:
  // the first-dispatched workgroups take them)
  for (int tile = first < 0 ? (int)blockIdx.x : first; tile < fold_tiles(a); tile += gridDim.x) {
    FoldOps<NW> f;
    fold_issue<NW>(a, tile, f);
    fold_mma<NW>(f, part);
    __syncthreads();
    fold_reduce(a, tile, part);
    __syncthreads();
  }
}

template <int D, bool QKV, bool IMG = false, int NW = WPB, bool TS = false, bool TR = true, bool LEAN = false>
__device__ __forceinline__ void attn16_fwd_body(const AttnArgs& a) {
  constexpr int LD = D + 8, NK = D / 32, NT = D / 16;
  // One LDS block carved into the kernel's buffers; the per-wave V / O tiles and the X tiles come
  // first and back to back, so the prologue can stage W_h through all three at once.
  //   vt, ot  [NW][16 * LD] bf16: per-wave V^T / O tiles
  //   xs      [2][NW][16 * LDX] bf16 (fused QKV): room for W_h's staging in the prologue (once the
  //           X tiles of the image mode's workgroup-wide build, which read_x replaced)
  //   zpart   [2][NW][16] fp32: fused pooled fc_o partial logits, double-buffered
  //   ztp     [2][NW][16 * 16] fp32: per-token fused fc_o z tiles per head, double-buffered
  //   imgs    [2][kImgPieces * 256] fp32 (image mode): the NW / Hl images of an iteration,
  //           double-buffered, padded to whole 1-KiB LDS-DMA pieces
  //   tsb     [NW][kTStamps] u64: diagnostic phase stamps
  constexpr int LDX = 88;
  constexpr int kImgPieces = (NW * 784 * 4 + 1023) / 1024;
  constexpr int kVt = NW * 16 * LD * 2, kXs = QKV ? 2 * NW * 16 * LDX * 2 : 0;
  constexpr int kZpart = 2 * NW * 16 * 4, kZtp = 2 * NW * 256 * 4;
  constexpr int kImgs = IMG ? 2 * kImgPieces * 1024 : 0, kTsb = QKV ? NW * kTStamps * 8 : 0;
  constexpr int oVt = 0, oOt = oVt + kVt, oXs = oOt + kVt, oZpart = oXs + kXs, oZtp = oZpart + kZpart,
                oImgs = oZtp + kZtp, oTsb = oImgs + kImgs, kSmem = oTsb + kTsb;
  constexpr int kStageBytes = oZpart;  // vt | ot | xs: W_h's staging room in the prologue
  static_assert(!QKV || kStageBytes >= 16 * 16 * 17 * 4, "the fold tail's partial tiles fit the stage");
  static_assert(!QKV || kZpart + kZtp >= 16 * 16 * 17 * 4, "... and the z-tile region");
  static_assert(oXs % 16 == 0 && oImgs % 16 == 0 && oTsb % 16 == 0, "16-B aligned LDS carve");
  __shared__ __attribute__((aligned(16))) char smem[kSmem];
  auto vt = reinterpret_cast<uint16_t(*)[16 * LD]>(smem + oVt);
  auto ot = reinterpret_cast<uint16_t(*)[16 * LD]>(smem + oOt);
  auto zpart = reinterpret_cast<float(*)[NW][16]>(smem + oZpart);
  auto ztp = reinterpret_cast<float(*)[NW][16 * 16]>(smem + oZtp);
  auto imgs = reinterpret_cast<float(*)[kImgPieces * 256]>(smem + oImgs);
  static_assert(!IMG || 2 * kImgPieces * 256 >= 16 * 16 * 17, "fold_tail reuses the image buffers");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int S = a.S, HD = a.Hl * D, npairs = a.B * a.Hl;
  const float inv_s = 1.f / (float)S;  // (fused path: means as multiplies)
  // diagnostic phase stamps (a.tstamp): shader clock per phase, lane 0 of each wave, into LDS
  auto tsb = reinterpret_cast<unsigned long long(*)[kTStamps]>(smem + oTsb);
  // (TS: the diagnostic instantiation; the production kernel carries no stamp code at all.
  // TR = false: the inference instantiation -- no lse / qkv / X-row / pool stores in its code)
  const bool tsr = TS && QKV && a.tstamp != nullptr;
  auto stamp = [&](int k) {
    if constexpr (QKV) {
      if (tsr) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (lane == 0 && k < kTStamps) tsb[wave][k] = t;
      }
    }
  };
  if constexpr (QKV) {
    // Touch every 64-B line of the argument block at once.  The prologue's argument reads are
    // spread over branches (fc_o bias, fold, image mode, ...), so the compiler waits on them in
    // ~10 batches; when the block is not in the scalar cache each batch was a full round trip to
    // the kernarg segment before any real work (profiles/r6_attn).  One round trip instead.
    const uint32_t __attribute__((address_space(4)))* kp =
        (const uint32_t __attribute__((address_space(4)))*)__builtin_amdgcn_kernarg_segment_ptr();
    static_assert(sizeof(AttnArgs) <= 8 * 64, "kernarg touch: 8 lines");
    asm volatile("" ::"s"(kp[0]), "s"(kp[16]), "s"(kp[32]), "s"(kp[48]), "s"(kp[64]), "s"(kp[80]), "s"(kp[96]),
                 "s"(kp[112]));
  }
  if (tsr && lane < kTStamps) tsb[wave][lane] = 0ull;  // (slots a short wave never reaches read 0)
  stamp(0);
  int itn = 0;  // iteration count (stamps 2 + 5 j .. 6 + 5 j, j < 4)
  // fused QKV: Hl | 4, so pair -> (sequence, head) is a shift and a mask, not a division
  const int lhl = a.Hl == 4 ? 2 : a.Hl == 2 ? 1 : 0;
  auto div_hl = [&](int x) { return QKV ? x >> lhl : x / a.Hl; };
  auto mod_hl = [&](int x) { return QKV ? x & (a.Hl - 1) : x % a.Hl; };
  // per-token fc_o: z rows stored (ztok), pushed (zrows), or -- fused QKV only -- reduced to
  // their mean over the S tokens in-kernel (zp: the local TP = 1 form, z never stored)
  const bool tok = a.ztok || a.zrows || (QKV && a.zp);
  uint16_t* V = vt[wave];
  uint16_t* O = ot[wave];
  // workgroup-uniform trip count (the fused fc_o reduces across the waves of an iteration);
  // with Hl | NW the Hl heads of a sequence are consecutive waves of one workgroup
  // fused fc_o: with Hl | NW this wave always serves head h = wave % Hl, so its W_o
  // entries (classes 4g..4g+3, features 16nt + c) are loaded once, packed as bf16 pairs
  uint32_t wpk[NT][2];
  if (!QKV && a.zp) {
    const int hw = mod_hl(wave);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        uint32_t lo = 0, hi = 0;
        const uint16_t* w = a.wo + (size_t)(4 * g + 2 * q) * a.ld_wo + hw * D + 16 * nt + c;
        if (4 * g + 2 * q < a.n_out) lo = w[0];
        if (4 * g + 2 * q + 1 < a.n_out) hi = w[a.ld_wo];
        wpk[nt][q] = lo | (hi << 16);
      }
  }
  // per-token fused fc_o: B operand of z = O . W_o^T -- lane (c, g) holds class c, this
  // wave's head features 32kk + 8g .. +7 (loaded once; classes >= n_out read as zero)
  bf16x8 wb[QKV ? 1 : NK];
  // fused QKV: z comes from the transposed O accumulators (features on the K axis), so W_o is
  // the B operand of the 16x16x16 MFMA -- lane (c, g): class c, features 16 nt + 4 g .. +3
  s4 wo16[QKV ? NT : 1];
  if (tok) {
    const int hw = mod_hl(wave);
    if constexpr (QKV) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        wo16[nt] = ld_s4(a.wo + (size_t)c * a.ld_wo + hw * D + 16 * nt + 4 * g, c < a.n_out);
    } else {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk)
        wb[kk] = ld_row16(a.wo + (size_t)c * a.ld_wo + hw * D + 32 * kk + 8 * g, c < a.n_out);
    }
  }
  // the workgroup's pair blocks (NW consecutive pairs each): grid-stride, except with the weight
  // fold at the start (pipelined plan) where a fold-owning workgroup (the first F) stops after kf
  // rounds and the others share the rest -- the fold costs ~1.5 iterations (profiles/r6_attn), so
  // at H = 2 (2 rounds) the fold owners' extra work no longer sets the kernel's length
  const int nblk = (npairs + NW - 1) / NW, G = gridDim.x, wg = blockIdx.x;
  int kf = 0x7fffffff, F = 0;
  if constexpr (QKV && IMG) {
    if (a.fold_sched > 0 && a.fold_out && a.fold_at_start && a.ld_wq == 72 && HD * 144 <= kStageBytes) {
      F = min(fold_tiles(a), G);
      if (F < G) kf = a.fold_sched - 1;
    }
  }
  auto blk = [&](int i) {  // this workgroup's i-th block; >= nblk: none (monotone in i)
    return i < kf ? wg + i * G : (wg < F ? nblk : kf * G + (wg - F) + (i - kf) * (G - F));
  };
  if constexpr (QKV && IMG) {
    // a fold-only workgroup (the grid widened by the fold's tiles, kf = 0): its tile and out --
    // no W_h staging, no images, nothing the attention workgroups beside it need
    if (F > 0 && blk(0) >= nblk) {
      if ((int)blockIdx.x < fold_tiles(a)) {
        float* part = reinterpret_cast<float*>(smem + oZpart);
        FoldOps<NW> fo;
        fold_issue<NW>(a, blockIdx.x, fo);
        fold_mma<NW>(fo, part);
        __syncthreads();
        fold_reduce(a, blockIdx.x, part);
      }
      return;
    }
  }
  // the fc_o bias of this lane's epilogue classes (4 (lane & 3) .. +3), loaded once (the
  // compiler cannot hoist it past the loop's global stores)
  float bov[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int cls = (lane & 3) * 4 + r;
    bov[r] = (tok && a.bo && cls < a.n_out) ? a.bo[cls] : 0.f;
  }
  // fused QKV: W_h's rows as B operands (lane (c, g): feature 16 nt + c of q | k | v, depth
  // 32 kk + 8 g .. +7, tail 64 + 4 g .. +3; zero past kq) and the bias, loaded once
  constexpr int WS = QKV ? 3 : 1, WN = QKV ? NT : 1;
  bf16x8 wf[WS][WN][2];
  s4 wtl[WS][WN];
  int it = 0;    // iteration parity: double-buffered LDS (z tiles, images)
  bf16x8 xn[2];  // the next iteration's patch rows (lane (c, g): token c, depth 32 kk + 8 g ..)
  s4 xtn;
  // fused QKV bias: two spare depth columns kb, kb + 1 (kq <= 72) hold X = 1 and W = the fp32
  // bias split into bf16 hi + lo parts, so the bias rides in the MFMA's fp32 accumulation (to
  // ~2^-17 relative -- far below the bf16 rounding of q | k | v) instead of 12 per-tile loads
  const int kb = a.kq > 64 ? a.kq : 64, gb = (kb - 64) >> 2;
  auto load_x = [&](int p) {  // patch-row mode: the pair's X rows from global memory
    const bool ok = p < npairs && c < S;
    const uint16_t* row = a.xq + (size_t)(ok ? div_hl(p) * S + c : 0) * a.ld_xq;
    xn[0] = ld_row16(row + 8 * g, ok && 8 * g < a.kq);
    xn[1] = ld_row16(row + 32 + 8 * g, ok && 32 + 8 * g < a.kq);
    xtn = ld_s4(row + 64 + 4 * g, ok && 64 + 4 * g < a.kq);
    if (g == gb) {  // the bias columns kb, kb + 1 of X are ones
      xtn[0] = (short)0x3F80;
      xtn[1] = (short)0x3F80;
    }
  };
  // LDS-DMA of the images of the iteration starting at pair p0 into buffer buf: straight from
  // global memory into LDS, no VGPRs held; bytes past the batch read as zero (buffer bounds)
  auto stage_imgs = [&](int buf, int p0) {
    if constexpr (IMG) {
      const int nseq = div_hl(NW), pieces = (nseq * 784 * 4 + 1023) / 1024;
      // (the descriptor starts at the iteration's first image: the bounds check covers
      // voffset, so the batch end clips exactly)
      const int b0 = div_hl(p0);
      const Rsrc rs = make_rsrc(uniform_ptr(reinterpret_cast<char*>(const_cast<float*>(a.img + (size_t)b0 * 784))), (uint32_t)((size_t)(a.B - b0) * 784 * 4));
      for (int pc = wave; pc < pieces; pc += NW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs.r, (__attribute__((address_space(3))) void*)(imgs[buf] + pc * 256),
                                                 16, (pc * 64 + lane) * 16, 0, 0, 0);
    }
  };
  // image mode: the wave's own X fragments (lane (c, g): token c; columns 8 g .., 32 + 8 g ..,
  // 64 + 4 g ..) straight from its sequence's image in LDS buffer buf.  MNIST 28 x 28 with 7 x 7
  // patches (S = 16): token t = patch (t / 4, t % 4); column cc < 49 is pixel (cc / 7, cc % 7) of
  // the patch, 49 the embedding bias 1, 50 + t the position one-hot, the rest zero, plus the QKV
  // bias columns kb, kb + 1 -- k_patchify's rows, bitwise.  (Round 6 until now: the workgroup
  // built the iteration's X tiles in LDS and every wave read its rows back -- one build round
  // and its stores cost ~1 k shader clocks per iteration, profiles/r6_attn.)
  auto read_x = [&](int buf) {
    if constexpr (IMG) {
      const float* im = imgs[buf] + div_hl(wave) * 784 + (c >> 2) * 196 + (c & 3) * 7;
      auto chunk = [&](int c0) {  // columns c0 .. c0 + 7 (c0 < 49 or past the pixels)
        int pr = c0 / 7, pc = c0 - 7 * pr;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cc = c0 + j;
          const float px = im[cc < 49 ? pr * 28 + pc : 0];
          v[j] = fmaf(px, cc < 49 ? 1.f : 0.f, (cc == 49 || cc == 50 + c) ? 1.f : 0.f);
          const bool wrap = pc == 6;
          pc = wrap ? 0 : pc + 1;
          pr += wrap ? 1 : 0;
        }
        const u32x4 w = {pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7])};
        return __builtin_bit_cast(bf16x8, w);
      };
      xn[0] = chunk(8 * g);
      xn[1] = chunk(32 + 8 * g);
      // the tail (columns 64 + 4 g .. +3): the position one-hot of tokens 14 and 15, the bias columns
#pragma unroll
      for (int j = 0; j < 4; ++j) xtn[j] = (64 + 4 * g + j == 50 + c) ? (short)0x3F80 : (short)0;
      if (g == gb) {
        xtn[0] = (short)0x3F80;
        xtn[1] = (short)0x3F80;
      }
    }
  };
  if constexpr (QKV) {
    const int hw = mod_hl(wave);
    if constexpr (IMG) {
      // (a fold owner may have no block at all: kf = 0)
      if (blk(0) < nblk) stage_imgs(0, blk(0) * NW);
      if (blk(1) < nblk) stage_imgs(1, blk(1) * NW);
    }
    // every load first (the bias by every lane, unconditionally), every use after
    float bqv[3][NT];
#pragma unroll
    for (int sel = 0; sel < 3; ++sel)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bqv[sel][nt] = a.bq[sel * HD + hw * D + 16 * nt + c];
    // the next forward's weight fold (image mode, at the start): this workgroup's tile's operand
    // loads go out with the prologue's own; with W_h staged below, its MFMAs run after the same
    // wait, its partial tiles go to the z-tile region (free until the first iteration) and the
    // staging barrier doubles as the fold's -- one round trip for both
    // (LEAN instantiations are launched only for the staged layout: no other W_h path in their
    // code)
    const bool staged = LEAN || (a.ld_wq == 72 && HD * 144 <= kStageBytes);
    const bool fold_first = IMG && a.fold_out && a.fold_at_start;
    const bool fold_here = fold_first && staged && (int)blockIdx.x < fold_tiles(a);
    FoldOps<NW> fo;
    if constexpr (IMG) {
      if (fold_here) fold_issue<NW>(a, blockIdx.x, fo);
      else if (fold_first && !staged) fold_tail<NW>(a, reinterpret_cast<float*>(smem + oVt));
    }
    float* fold_part = reinterpret_cast<float*>(smem + oZpart);  // zpart | ztp: 16 * 16 * 17 floats
    // W_h staged ONCE per workgroup: the wave reading it from global memory itself made every
    // wave of the grid pull its head's 27.6 KiB through L2 at the same moment (57 MiB at
    // B = 2048: 9-12 k shader clocks of issue stalls per wave before any work, a third of the
    // kernel, profiles/r6_attn).  Per projection (q, k, v) the Hl local heads' rows -- one
    // contiguous HD x 144-B block when ld_wq = 72 -- go into the X tiles' LDS by LDS-DMA and every
    // wave reads its fragments from there: the grid's L2 traffic for W falls by the waves per
    // head of a workgroup (NW / Hl: 4 at TP = 2, 2 at TP = 1).
    const int selb = HD * 144;  // one projection's rows of every local head (ld_wq = 72)
    if (staged) {
      char* stg = smem + oVt;
      // as many projections per round as the V / O / X tiles hold: TP = 2 (HD = 128) all three at
      // once, TP = 1 (HD = 256) q | k then v -- every round one LDS-DMA latency and two barriers
      const int per_round = kStageBytes / selb;
      int done = 0, r0 = 0;  // end of the staged projections, first projection of the round
#pragma unroll
      for (int sel = 0; sel < 3; ++sel) {
        if (sel == done) {  // issue the round starting at this projection
          if (tsr && sel == 0) {  // (diagnostic only: the argument / bias / image loads alone)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp(28);
          }
          const int nsel = min(per_round, 3 - sel), bytes = nsel * selb, pieces = (bytes + 1023) / 1024;
          const Rsrc rs = make_rsrc(uniform_ptr(reinterpret_cast<char*>(const_cast<uint16_t*>(a.wq + (size_t)sel * HD * 72))),
                                    (uint32_t)bytes);
          for (int pc = wave; pc < pieces; pc += NW)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs.r, (__attribute__((address_space(3))) void*)(stg + pc * 1024), 16,
                                                     (pc * 64 + lane) * 16, 0, 0, 0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (sel == 0) stamp(29);  // this wave's W_h DMA landed
          if (IMG && sel == 0 && fold_here) fold_mma<NW>(fo, fold_part);
          __syncthreads();
          if (IMG && sel == 0 && fold_here) fold_reduce(a, blockIdx.x, fold_part);
          done = sel + nsel;
          r0 = sel;
        }
        const int slot = sel - r0;  // this projection's block in the stage
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint16_t* row = reinterpret_cast<const uint16_t*>(stg + (size_t)slot * selb) + (size_t)(hw * D + 16 * nt + c) * 72;
          wf[sel][nt][0] = 8 * g < a.kq ? *reinterpret_cast<const bf16x8*>(row + 8 * g) : bf16x8{};
          wf[sel][nt][1] = 32 + 8 * g < a.kq ? *reinterpret_cast<const bf16x8*>(row + 32 + 8 * g) : bf16x8{};
          wtl[sel][nt] = 64 + 4 * g < a.kq ? *reinterpret_cast<const s4*>(row + 64 + 4 * g) : s4{0, 0, 0, 0};
        }
        if (sel + 1 == done) __syncthreads();  // (the round's last projection read: the stage is free)
      }

    } else {
#pragma unroll
      for (int sel = 0; sel < 3; ++sel)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint16_t* w = a.wq + (size_t)(sel * HD + hw * D + 16 * nt + c) * a.ld_wq;
          wf[sel][nt][0] = ld_row16(w + 8 * g, 8 * g < a.kq);
          wf[sel][nt][1] = ld_row16(w + 32 + 8 * g, 32 + 8 * g < a.kq);
          wtl[sel][nt] = ld_s4(w + 64 + 4 * g, 64 + 4 * g < a.kq);
        }
    }
    stamp(24);  // every W_h load issued (staged: and its fragments read back)
#pragma unroll
    for (int sel = 0; sel < 3; ++sel)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float bias = bqv[sel][nt];
        const uint32_t hi = f32_to_bf16_bits(bias);
        const short lo = (short)f32_to_bf16_bits(bias - __uint_as_float(hi << 16));
        wtl[sel][nt][0] = g == gb ? (short)hi : wtl[sel][nt][0];
        wtl[sel][nt][1] = g == gb ? lo : wtl[sel][nt][1];
      }
    stamp(25);  // W_h's tail fragments and biases arrived
    if constexpr (!IMG) load_x(blk(0) * NW + wave);
    if constexpr (IMG) {
      // images two iterations deep: the first two (their DMA issued before W_h's), the first
      // one's X fragments read once they are visible -- with W_h staged, every wave waited for
      // all its loads (images included) before the staging barrier, so they are already
      if (!staged) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(26);  // every W_h load and both images' DMA landed
        __syncthreads();
      } else {
        stamp(26);
      }
      read_x(0);
      // every wave's reads of buffer 0 done before any wave's first loop DMA refills it (the
      // images of the third block; an L2-resident image lands within a few hundred clocks)
      if (blk(2) < nblk) __syncthreads();
      stamp(27);
    }
  }
  stamp(1);
  for (int bi = blk(0); bi < nblk; bi = blk(itn + 1), it ^= 1, ++itn) {
   const int base = bi * NW;
   const int pr = base + wave;
   const int sj = itn < 4 ? 2 + 5 * itn : kTStamps;  // this iteration's stamp slots
   bf16x8 xr[2];
   s4 xt;
   if constexpr (QKV) {
    // (image mode: xn holds this iteration's fragments, read at the end of the previous one)
    if constexpr (IMG) {
      // the images of the iteration after next, into the buffer this iteration's X was read
      // from -- by every wave before the last barrier (the body issues no further global
      // loads, so nothing waits on this DMA before the epilogue's vmcnt(0); the trip count is
      // workgroup-uniform, so every piece is issued)
      if (blk(itn + 2) < nblk) stage_imgs(it, blk(itn + 2) * NW);
    }
    xr[0] = xn[0];
    xr[1] = xn[1];
    xt = xtn;
    if constexpr (!IMG) load_x(blk(itn + 1) * NW + wave);
   }
   stamp(sj);
   if (pr < npairs) {
    const int b = div_hl(pr), h = mod_hl(pr);
    bf16x8 qr[NK], kr[NK];
    if constexpr (QKV) {
      // sel's [16 tokens][D] block of X W_h^T + b (the bias via the tail's bias columns),
      // rounded to bf16, into tile T -- computed transposed, (W_h X^T), so a lane's accumulator
      // holds 4 consecutive features of one token: 2 packed conversions + one 8-B LDS store
      // per 16 x 16 tile instead of 4 + 4 2-B stores.  (The first version re-read the bias per
      // tile: flat loads + vmcnt(0) waits that also drained the X prefetch, 12 per pair.)
      auto proj = [&](int sel, uint16_t* T) {
#pragma unroll
        for (int nt = 0; nt < NT; nt += 2) {  // two tiles in flight: the MFMAs overlap the conversions
          // (the 16x16x16 tail gets its own accumulator: chaining it onto the 16x16x32
          // accumulator lost rows -- the compiler emits no wait states for that srcC hazard)
          f4 tl[2], acc[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            tl[u] = mma16(wtl[sel][nt + u], xt, f4{0.f, 0.f, 0.f, 0.f});
            acc[u] = mma32(wf[sel][nt + u][0], xr[0], f4{0.f, 0.f, 0.f, 0.f});
          }
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[u] = mma32(wf[sel][nt + u][1], xr[1], acc[u]);  // [feature 16 nt + 4g + r][token c]
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const uint2 pk = {pk_bf16(acc[u][0] + tl[u][0], acc[u][1] + tl[u][1]),
                              pk_bf16(acc[u][2] + tl[u][2], acc[u][3] + tl[u][3])};
            *reinterpret_cast<uint2*>(T + c * LD + 16 * (nt + u) + 4 * g) = pk;
          }
        }
      };
      if (TR && IMG && a.xq_out && h == 0 && c < S) {  // the patch rows, for the backward (one head's wave)
        uint16_t* xo = a.xq_out + (size_t)(b * S + c) * a.ld_xq;
        if (8 * g < a.kq) *reinterpret_cast<bf16x8*>(xo + 8 * g) = xr[0];
        if (32 + 8 * g < a.kq) *reinterpret_cast<bf16x8*>(xo + 32 + 8 * g) = xr[1];
        if (64 + 4 * g < a.kq) *reinterpret_cast<s4*>(xo + 64 + 4 * g) = xt;
      }
      proj(0, O);
      proj(1, V);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        qr[kk] = *reinterpret_cast<const bf16x8*>(O + c * LD + 32 * kk + 8 * g);
        kr[kk] = *reinterpret_cast<const bf16x8*>(V + c * LD + 32 * kk + 8 * g);
      }
      uint16_t* qo = TR && a.qkv_out ? a.qkv_out + (size_t)b * S * a.ld_qkv + h * D : nullptr;
      if (qo) {
        rows_out<D, LD>(O, qo, a.ld_qkv, S, lane);
        rows_out<D, LD>(V, qo + HD, a.ld_qkv, S, lane);
      }
      __builtin_amdgcn_wave_barrier();
      // v un-transposed (acc[r] = v[token 4g + r][feature 16 nt + c]) into the V^T tile
      // ([D features][16 tokens], one 8-B store per lane per tile): the PV MFMA's operand
      // (keys 4g .. 4g+3 of one feature) is then ONE 8-B LDS read instead of four 2-B reads.
      // For a backward, v also goes row-major into the (free) O tile for the qkv store.
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const f4 tl = mma16(xt, wtl[2][nt], f4{0.f, 0.f, 0.f, 0.f});
        f4 acc = mma32(xr[0], wf[2][nt][0], f4{0.f, 0.f, 0.f, 0.f});
        acc = mma32(xr[1], wf[2][nt][1], acc);
        const uint2 pk = {pk_bf16(acc[0] + tl[0], acc[1] + tl[1]), pk_bf16(acc[2] + tl[2], acc[3] + tl[3])};
        *reinterpret_cast<uint2*>(V + (16 * nt + c) * 16 + 4 * g) = pk;
        if (qo) {
          O[(4 * g + 0) * LD + 16 * nt + c] = (uint16_t)(pk.x & 0xffffu);
          O[(4 * g + 1) * LD + 16 * nt + c] = (uint16_t)(pk.x >> 16);
          O[(4 * g + 2) * LD + 16 * nt + c] = (uint16_t)(pk.y & 0xffffu);
          O[(4 * g + 3) * LD + 16 * nt + c] = (uint16_t)(pk.y >> 16);
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (qo) rows_out<D, LD>(O, qo + 2 * HD, a.ld_qkv, S, lane);
      stamp(sj + 1);
    } else {
      const uint16_t* qb = a.qkv + (size_t)b * S * a.ld_qkv + h * D;
      bf16x8 vr[NK];
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const size_t off = (size_t)c * a.ld_qkv + 32 * kk + 8 * g;
        qr[kk] = ld_row16(qb + off, c < S);
        kr[kk] = ld_row16(qb + HD + off, c < S);
        vr[kk] = ld_row16(qb + 2 * HD + off, c < S);
      }
      put_rows<D, LD>(V, vr, lane);
    }
    f4 st = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) st = mma32(kr[kk], qr[kk], st);  // S^T[j = 4g + r][i = c]
    float x[4], m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[r] = (4 * g + r < S) ? st[r] * a.scale : -INFINITY;
      m = fmaxf(m, x[r]);
    }
    m = pair32_max(pair16_max(m));
    float e[4], s = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      e[r] = __expf(x[r] - m);
      s += e[r];
    }
    s = pair32_sum(pair16_sum(s));
    // (fused path: the hardware reciprocal -- the precise division is ~10 VALU ops, and the
    // probabilities are rounded to bf16 right after)
    const float inv = QKV ? __builtin_amdgcn_rcpf(s) : 1.f / s;
    if (TR && a.lse && g == 0 && c < S) a.lse[(size_t)pr * S + c] = m + __logf(s);
    const s4 pa = pack4(e[0] * inv, e[1] * inv, e[2] * inv, e[3] * inv);  // A[i = c][j = 4g + jj]
    __builtin_amdgcn_wave_barrier();
    if constexpr (QKV) {
      // O^T = V^T P^T: ot[nt][r] = O[query c][feature 16 nt + 4g + r] -- features on the MFMA
      // K axis, so z = bf16(O) W_o^T chains straight from the registers (no LDS round trip)
      f4 ot[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        ot[nt] = mma16(*reinterpret_cast<const s4*>(V + (16 * nt + c) * 16 + 4 * g), pa, f4{0.f, 0.f, 0.f, 0.f});
      f4 zt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) zt = mma16(pack4(ot[nt][0], ot[nt][1], ot[nt][2], ot[nt][3]), wo16[nt], zt);
#pragma unroll
      for (int r = 0; r < 4; ++r) ztp[it][wave][(4 * g + r) * 16 + c] = zt[r];  // z[i = 4g + r][cls = c]
      stamp(sj + 2);
      if (TR && a.pool) {
        // pool[f] = mean over the S queries of O[i][f]: recompute O un-transposed (4 more
        // 16x16x16 MFMAs, one tile live at a time) so the column sum is 4 adds + 2 shuffles per
        // tile -- and bitwise the unfused kernel's pool.  (A 15-shuffle butterfly over the
        // transposed accumulators pushed the kernel past 256 VGPRs.)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const f4 on = mma16(pa, *reinterpret_cast<const s4*>(V + (16 * nt + c) * 16 + 4 * g), f4{0.f, 0.f, 0.f, 0.f});
          float cs = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) cs += (4 * g + r < S) ? on[r] : 0.f;
          cs = pair32_sum(pair16_sum(cs));
          if (g == 0) a.pool[(size_t)b * a.ld_pool + h * D + 16 * nt + c] = (uint16_t)f32_to_bf16_bits(cs * inv_s);
        }
      }
    } else {
    f4 o[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) o[nt] = mma16(pa, tile_b<LD>(V, g, 16 * nt + c), f4{0.f, 0.f, 0.f, 0.f});
    if (a.pool) {
      // pooled features 16nt + c; with the fused fc_o each one is folded into this head's
      // share of the logits right away (lane (c, g) takes classes 4g..4g+3), keeping few
      // registers live
      float zacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        float cs = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) cs += (4 * g + r < S) ? o[nt][r] : 0.f;
        cs = pair32_sum(pair16_sum(cs));
        const uint32_t pb = f32_to_bf16_bits(cs / (float)S);
        if (g == 0) a.pool[(size_t)b * a.ld_pool + h * D + 16 * nt + c] = (uint16_t)pb;
        if (!QKV && a.zp) {
          const float pv = __uint_as_float(pb << 16);  // the bf16 value a separate fc_o GEMM would read
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            zacc[2 * q] += pv * bf16_lo(wpk[nt][q]);
            zacc[2 * q + 1] += pv * bf16_hi(wpk[nt][q]);
          }
        }
      }
      if (!QKV && a.zp) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float acc = zacc[j];
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) acc += __shfl_xor(acc, off);
          if (c == 0) zpart[it][wave][4 * g + j] = acc;
        }
      }
    }
    if (tok) {
      // z[i][cls] over this head's features on the MFMA: A = bf16(O) rows (the values a
      // separate fc_o GEMM would read) from this wave's LDS tile, B = W_o in registers;
      // the accumulator holds z[i = 4g + r][cls = c]
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) O[(4 * g + r) * LD + 16 * nt + c] = (uint16_t)f32_to_bf16_bits(o[nt][r]);
      __builtin_amdgcn_wave_barrier();
      f4 zt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) zt = mma32(*reinterpret_cast<const bf16x8*>(O + c * LD + 32 * kk + 8 * g), wb[kk], zt);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 4; ++r) ztp[it][wave][(4 * g + r) * 16 + c] = zt[r];
    }
    if (a.o) store_tile<D, LD>(O, o, 1.f, a.o + (size_t)b * S * a.ld_o + h * D, a.ld_o, S, lane);
    }  // !QKV
   }
   if (tok) {
    // the Hl heads of each sequence of this iteration (consecutive waves, Hl | NW), summed in
    // head order, + the bias.  Wave s writes sequence s (waves s >= NW / Hl idle): lane l =
    // (token l >> 2, classes 4 (l & 3) .. +3), one 16-B store per lane, a sequence's S x 16
    // fp32 rows as whole lines
    if constexpr (IMG) {
      // the next iteration's X, from images visible since the last barrier (read before the
      // barrier below: the next iteration's DMA overwrites this buffer); then this wave's DMA
      // of the images two iterations ahead has landed (visible to every wave after the barrier)
      if (blk(itn + 1) < nblk) read_x(it ^ 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    stamp(sj + 3);
    __syncthreads();  // (the next iteration writes the other buffer)
    const int i = lane >> 2, q = (lane & 3) * 4, w = wave * a.Hl;
    const int prw = base + w;
    if (w < NW && prw < npairs) {
      const int b = div_hl(prw);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = bov[r];
      float z4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < a.Hl; ++k) {
        const float4 x = *reinterpret_cast<const float4*>(&ztp[it][w + k][i * 16 + q]);
        z4[0] += x.x; z4[1] += x.y; z4[2] += x.z; z4[3] += x.w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = z4[r] + v[r];
      const u32x4 pk = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
      const size_t row0 = (size_t)b * S;  // the sequence's first row
      if (i < S) {
        if (a.zrows) {
          // zrows % S == 0: the whole sequence lies in block j (wave-uniform); rank j's inbox
          // slot over xGMI, stored write-through (sc0 sc1) like every collective store
          const int j = __builtin_amdgcn_readfirstlane((int)(row0 / a.zrows));
          char* seq = reinterpret_cast<char*>(a.zpush[j] + (row0 - (size_t)j * a.zrows) * a.ld_zt);
          const Rsrc rs = make_rsrc(uniform_ptr(seq), (uint32_t)(S * a.ld_zt * 4));
          __builtin_amdgcn_raw_buffer_store_b128(pk, rs.r, (uint32_t)((i * a.ld_zt + q) * 4), 0, kStorePolicy);
        } else if (a.ztok) {
          *reinterpret_cast<u32x4*>(a.ztok + (row0 + i) * a.ld_zt + q) = pk;
        }
      }
      if (QKV && a.zp) {  // logits = mean over the S tokens (lanes 4 i + (q / 4))
        float m[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          m[r] = i < S ? v[r] : 0.f;
          // the row's 4 tokens of this class group (lanes 4 apart in a 16-lane row) by DPP row
          // rotations of 4, 8 and 12 (the other three, whichever way the rotation runs), not a
          // ds_bpermute round trip per __shfl_xor
          m[r] = ((m[r] + row_ror<4>(m[r])) + row_ror<12>(m[r])) + row_ror<8>(m[r]);
          m[r] = pair32_sum(pair16_sum(m[r]));
        }
        if (i == 0) {
          *reinterpret_cast<float4*>(a.zp + (size_t)b * a.ld_zp + q) =
              float4{m[0] * inv_s, m[1] * inv_s, m[2] * inv_s, m[3] * inv_s};
        }
      }
    }
    stamp(sj + 4);
   }
   if (!QKV && a.zp) {  // sum the Hl heads of each sequence in rank order (deterministic) and add the bias
    __syncthreads();  // (the next iteration writes the other buffer: one barrier per iteration)
    const int t = threadIdx.x, w = t >> 4, cls = t & 15, prw = base + w;
    if (t < NW * 16 && prw < npairs && mod_hl(prw) == 0 && cls < a.n_out) {
      float acc = 0.f;
      for (int k = 0; k < a.Hl; ++k) acc += zpart[it][w + k][cls];
      if (a.bo) acc += a.bo[cls];
      a.zp[(size_t)div_hl(prw) * a.ld_zp + cls] = acc;
    }
   }
  }
  if constexpr (QKV && IMG) {
    // the next forward's weight fold in the images' LDS (every DMA into it has landed: each
    // trip ends with vmcnt(0) and a barrier, and the trip count is workgroup-uniform)
    if (!LEAN && a.fold_out && !a.fold_at_start) {  // (LEAN: launched only with the fold at the start)
      __syncthreads();
      fold_tail<NW>(a, &imgs[0][0]);
    }  // (fold at the start: one tile per workgroup at most -- launch_qkv_fwd_mfma moves a
       // larger fold to the standalone kernel)
  }
  if constexpr (QKV) {
    if (tsr) {
      stamp(kTStamps - 1);
      __builtin_amdgcn_wave_barrier();
      if (lane < kTStamps) a.tstamp[((size_t)blockIdx.x * NW + wave) * kTStamps + lane] = tsb[wave][lane];
    }
  }
}


template <int D>
__global__ void __launch_bounds__(256) k_attn16_fwd(AttnArgs a) {
  attn16_fwd_body<D, false>(a);
}

// One workgroup of kQkvWaves waves per CU (two per SIMD): <= 256 VGPRs a wave, W_h's fragments
// included; the waves of a workgroup share its staged W_h (see attn16_fwd_body).
constexpr int kQkvWaves = 8;
template <int D, bool IMG, bool TS, bool TR, bool LEAN>
__global__ void __launch_bounds__(64 * kQkvWaves) __attribute__((amdgpu_waves_per_eu(2))) k_qkv_attn16_fwd(AttnArgs a) {
  attn16_fwd_body<D, true, IMG, kQkvWaves, TS, TR, LEAN>(a);
}

template <int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D == 128 ? 2 : 4))) k_attn16_bwd(AttnArgs a) {
  constexpr int LD = D + 8, NK = D / 32, NT = D / 16, TILE = 16 * LD;
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  uint16_t* Qt = sm + wave * 4 * TILE;
  uint16_t* Kt = Qt + TILE;
  uint16_t* Dt = Kt + TILE;
  uint16_t* Ot = Dt + TILE;
  const int S = a.S, HD = a.Hl * D;
  float bq[NT], bk[NT], bv[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bq[nt] = bk[nt] = bv[nt] = 0.f;
  // workgroup k owns head h = k % Hl; its waves stride over the batch, so the
  // bias column sums of the 4 waves meet in LDS and leave with one atomic per
  // column per workgroup (per-wave atomics on the same 3*D addresses contend)
  const int h = blockIdx.x % a.Hl, nbh = gridDim.x / a.Hl;
  // fused pooled fc_o input gradient: this head's slice of W_o, fp32, for every sequence
  // (bf16, 2 KiB at D = 64: the workgroup stays within 40 KiB of LDS, 4 per CU)
  __shared__ uint16_t wos[16 * D];
  if (a.dz) {
    for (int i = threadIdx.x; i < 16 * D; i += blockDim.x) {
      const int cls = i / D;
      wos[i] = cls < a.n_out ? a.wo[(size_t)cls * a.ld_wo + h * D + i % D] : (uint16_t)0;
    }
    __syncthreads();
  }
  for (int b = (blockIdx.x / a.Hl) * WPB + wave; b < a.B; b += nbh * WPB) {
    const int pr = b * a.Hl + h;
    const uint16_t* qb = a.qkv + (size_t)b * S * a.ld_qkv + h * D;
    bf16x8 qr[NK], kr[NK], vr[NK], dr[NK];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const size_t off = (size_t)c * a.ld_qkv + 32 * kk + 8 * g;
      qr[kk] = ld_row16(qb + off, c < S);
      kr[kk] = ld_row16(qb + HD + off, c < S);
      vr[kk] = ld_row16(qb + 2 * HD + off, c < S);
    }
    if (a.dz) {
      // dO row (every one of the S rows) = dz_scale * dz[b] . W_o[:, h*D .. h*D + D),
      // rounded to bf16 like the separate dpool GEMM's output
      // the dz row is wave-uniform: keep its 8 words in scalar registers
      const uint32_t* zrow = reinterpret_cast<const uint32_t*>(a.dz + (size_t)__builtin_amdgcn_readfirstlane(b) * a.ld_dz);
      uint32_t zw[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) zw[q] = __builtin_amdgcn_readfirstlane(zrow[q]);
      for (int col = lane; col < D; col += 64) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          v += bf16_lo(zw[q]) * __uint_as_float((uint32_t)wos[(2 * q) * D + col] << 16);
          v += bf16_hi(zw[q]) * __uint_as_float((uint32_t)wos[(2 * q + 1) * D + col] << 16);
        }
        Dt[col] = (uint16_t)f32_to_bf16_bits(v * a.dz_scale);  // row 0 of this wave's dO tile
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) dr[kk] = ld_row16(Dt + 32 * kk + 8 * g, c < S);
      __builtin_amdgcn_wave_barrier();  // put_rows below rewrites the tile
    } else {
      const uint16_t* db = a.dout + (size_t)b * a.dout_bstride + h * D;
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) dr[kk] = ld_row16(db + (size_t)c * a.dout_rstride + 32 * kk + 8 * g, c < S);
    }
    put_rows<D, LD>(Qt, qr, lane);
    put_rows<D, LD>(Kt, kr, lane);
    put_rows<D, LD>(Dt, dr, lane);
    const float* lse = a.lse + (size_t)pr * S;
    const float lse_c = c < S ? lse[c] : 0.f;
    float lse_r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lse_r[r] = (4 * g + r < S) ? lse[4 * g + r] : 0.f;
    f4 sT = {0.f, 0.f, 0.f, 0.f}, sM = sT, dpT = sT, dpM = sT;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      sT = mma32(kr[kk], qr[kk], sT);    // S^T[j = 4g + r][i = c]
      sM = mma32(qr[kk], kr[kk], sM);    // S[i = 4g + r][j = c]
      dpT = mma32(vr[kk], dr[kk], dpT);  // dP^T[j = 4g + r][i = c]
      dpM = mma32(dr[kk], vr[kk], dpM);  // dP[i = 4g + r][j = c]
    }
    // delta_i = sum_d dO[i][d] O[i][d] = sum_j P[i][j] dP[i][j]: from the probabilities
    // and dP already in registers, so O is never read (and need not be stored)
    float P[4], PT[4], dS[4], dST[4];
    float dl = 0.f, dl_r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = (4 * g + r < S) && (c < S);
      PT[r] = ok ? __expf(sT[r] * a.scale - lse_c) : 0.f;
      P[r] = ok ? __expf(sM[r] * a.scale - lse_r[r]) : 0.f;
      dl += PT[r] * dpT[r];          // row i = c: keys j = 4g + r in registers ...
      dl_r[r] = P[r] * dpM[r];       // row i = 4g + r: keys j = c on the lanes ...
    }
    dl = pair32_sum(pair16_sum(dl));  // ... and across the four lane groups
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) dl_r[r] += __shfl_xor(dl_r[r], o);  // ... and across the 16 lanes
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dST[r] = PT[r] * (dpT[r] - dl);
      dS[r] = P[r] * (dpM[r] - dl_r[r]);
    }
    __builtin_amdgcn_wave_barrier();
    const s4 aP = pack4(P[0], P[1], P[2], P[3]);        // A[j = c][i = 4g + jj] = P^T
    const s4 aDS = pack4(dS[0], dS[1], dS[2], dS[3]);   // A[j = c][i = 4g + jj] = dS^T
    const s4 aDST = pack4(dST[0], dST[1], dST[2], dST[3]);  // A[i = c][j = 4g + jj] = dS
    f4 acc[NT];
    uint16_t* gq = a.dqkv + (size_t)b * S * a.ld_qkv + h * D;
    // dV = P^T dO
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      acc[nt] = mma16(aP, tile_b<LD>(Dt, g, 16 * nt + c), f4{0.f, 0.f, 0.f, 0.f});
      bv[nt] += acc[nt][0] + acc[nt][1] + acc[nt][2] + acc[nt][3];
    }
    store_tile<D, LD>(Ot, acc, 1.f, gq + 2 * HD, a.ld_qkv, S, lane);
    // dK = scale dS^T Q
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      acc[nt] = mma16(aDS, tile_b<LD>(Qt, g, 16 * nt + c), f4{0.f, 0.f, 0.f, 0.f});
      bk[nt] += a.scale * (acc[nt][0] + acc[nt][1] + acc[nt][2] + acc[nt][3]);
    }
    store_tile<D, LD>(Ot, acc, a.scale, gq + HD, a.ld_qkv, S, lane);
    // dQ = scale dS K
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      acc[nt] = mma16(aDST, tile_b<LD>(Kt, g, 16 * nt + c), f4{0.f, 0.f, 0.f, 0.f});
      bq[nt] += a.scale * (acc[nt][0] + acc[nt][1] + acc[nt][2] + acc[nt][3]);
    }
    store_tile<D, LD>(Ot, acc, a.scale, gq, a.ld_qkv, S, lane);
  }
  if (a.dbias) {
    float* red = reinterpret_cast<float*>(sm);  // reuse the tiles: [WPB][3][D] fp32
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float q = bq[nt], k = bk[nt], v = bv[nt];
      q = pair32_sum(pair16_sum(q));
      k = pair32_sum(pair16_sum(k));
      v = pair32_sum(pair16_sum(v));
      if (g == 0) {
        red[(wave * 3 + 0) * D + 16 * nt + c] = q;
        red[(wave * 3 + 1) * D + 16 * nt + c] = k;
        red[(wave * 3 + 2) * D + 16 * nt + c] = v;
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * D; i += blockDim.x) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < WPB; ++w) acc += red[w * 3 * D + i];
      atomicAdd(a.dbias + (i / D) * HD + h * D + i % D, acc);
    }
  }
}

template <int D>
constexpr size_t bwd_lds_bytes() {
  return (size_t)WPB * 4 * 16 * (D + 8) * sizeof(uint16_t);
}

int grid_for(int npairs, int cap, int nw = WPB) { return std::max(1, std::min((npairs + nw - 1) / nw, cap)); }

}  // namespace

bool mfma_supported(const AttnArgs& a, bool bwd) {
  if (a.S < 1 || a.S > 16 || !(a.D == 32 || a.D == 64 || a.D == 128)) return false;
  if (a.ld_qkv % 8 || a.ld_o % 8 || ((uint64_t)a.qkv % 16) || ((uint64_t)a.o % 16)) return false;
  if (bwd && (a.dout_bstride % 8 || a.dout_rstride % 8 || ((uint64_t)a.dout % 16) || ((uint64_t)a.dqkv % 16))) return false;
  return true;
}

void launch_fwd_mfma(const AttnArgs& a, hipStream_t stream) {
  const int grid = grid_for(a.B * a.Hl, 4096);
  if (a.D == 32) hipLaunchKernelGGL(k_attn16_fwd<32>, dim3(grid), dim3(256), 0, stream, a);
  else if (a.D == 64) hipLaunchKernelGGL(k_attn16_fwd<64>, dim3(grid), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(k_attn16_fwd<128>, dim3(grid), dim3(256), 0, stream, a);
}

// persistent: one 8-wave workgroup per CU (W_h staged once per workgroup, held in registers by
// every wave); attn_set_qkv_grid / CCMPI_QKV_GRID
int g_qkv_grid_cap = std::getenv("CCMPI_QKV_GRID") ? std::atoi(std::getenv("CCMPI_QKV_GRID")) : 256;

// The in-kernel weight fold's cost in pair rounds of the fused forward (H = 2: ~3 us against
// ~2.1 us per round; H = 4: ~3.2 against ~2.7; profiles/r6_attn trace_v9_fold / trace_v12).
constexpr double kFoldRounds = 1.5;
int g_qkv_fold_sched = -1;  // -1: CCMPI_QKV_FOLD_SCHED (default on), 0: grid-stride always, 1: on
int g_qkv_fold_grid = 1;    // fold workgroups of their own on a grid with CUs to spare (0 when ranks share the GPU)

// AttnArgs::fold_sched for a launch of `grid` workgroups: the rounds kf of the fold-owning
// workgroups that minimise max(kf + fold, the others' rounds); 0 when grid-stride is as good
bool fold_sched_on() {
  if (g_qkv_fold_sched < 0) {
    const char* e = std::getenv("CCMPI_QKV_FOLD_SCHED");
    g_qkv_fold_sched = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  return g_qkv_fold_sched != 0;
}

int fold_sched_for(const AttnArgs& a, int grid) {
  if (!fold_sched_on() || !a.img || !a.fold_out || !a.fold_at_start) return 0;
  const int nblk = (a.B * a.Hl + kQkvWaves - 1) / kQkvWaves;
  const int F = std::min(((a.fold_R + 15) / 16) * ((a.fold_kp + 15) / 16), grid);
  if (F <= 0 || F >= grid) return 0;
  const int kstd = (nblk + grid - 1) / grid;
  double best = kstd + kFoldRounds;
  int bk = kstd;
  for (int kf = kstd - 1; kf >= 0; --kf) {
    const int rest = nblk - kf * grid;
    const int others = kf + (rest > 0 ? (rest + grid - F - 1) / (grid - F) : 0);
    const double cost = std::max(kf + kFoldRounds, (double)others);
    if (cost < best) {
      best = cost;
      bk = kf;
    }
  }
  return bk == kstd ? 0 : bk + 1;
}

template <bool TS, bool TR, bool LEAN>
void launch_qkv_variant(const AttnArgs& a, int grid, dim3 block, hipStream_t stream) {
  if (a.img) {
    if (a.D == 32) hipLaunchKernelGGL((k_qkv_attn16_fwd<32, true, TS, TR, LEAN>), dim3(grid), block, 0, stream, a);
    else hipLaunchKernelGGL((k_qkv_attn16_fwd<64, true, TS, TR, LEAN>), dim3(grid), block, 0, stream, a);
  } else {
    if (a.D == 32) hipLaunchKernelGGL((k_qkv_attn16_fwd<32, false, TS, TR, LEAN>), dim3(grid), block, 0, stream, a);
    else hipLaunchKernelGGL((k_qkv_attn16_fwd<64, false, TS, TR, LEAN>), dim3(grid), block, 0, stream, a);
  }
}

void launch_qkv_fwd_mfma(const AttnArgs& args, hipStream_t stream) {
  int grid = grid_for(args.B * args.Hl, g_qkv_grid_cap, kQkvWaves);
  const int fold_tiles_n = args.fold_out ? ((args.fold_R + 15) / 16) * ((args.fold_kp + 15) / 16) : 0;
  // a fold at the start on a grid with CUs to spare (a small per-rank batch -- DP4 x TP2 at 512
  // sequences is 128 blocks): the fold's tiles get workgroups of their own beside the attention
  // workgroups (fold_sched_for then gives them no pair block), instead of running before those
  // workgroups' only block
  // (not when ranks share the GPU, g_qkv_fold_grid = 0: their kernels already fill every CU)
  if (args.img && fold_tiles_n && args.fold_at_start && args.ld_wq == 72 && fold_sched_on() && g_qkv_fold_grid &&
      grid < g_qkv_grid_cap)
    grid = std::min(g_qkv_grid_cap, grid + fold_tiles_n);
  const dim3 block(64 * kQkvWaves);
  AttnArgs a = args;
  // more fold tiles than workgroups (small batches): the whole fold goes to the standalone
  // fp32-MFMA kernel after this one (bitwise the same; it writes the NEXT forward's W_eff, which
  // this kernel does not read), so the fused kernel carries one copy of the fold code, not two
  const bool fold_apart = a.fold_out && fold_tiles_n > grid;
  if (fold_apart) a.fold_out = nullptr;
  a.fold_sched = fold_sched_for(a, grid);
  // instantiations: TS = the phase-stamp diagnostic; TR = the training stores (lse, qkv, X rows,
  // pool) in the code; LEAN = W_h staged and any fold at the start, the only paths in the code
  // (the instruction cache: every byte of a path the kernel never takes still costs fetch time)
  const bool train = a.lse || a.qkv_out || a.xq_out || a.pool;
  const bool lean = a.ld_wq == 72 && (!a.fold_out || a.fold_at_start);
  if (a.tstamp) launch_qkv_variant<true, true, false>(a, grid, block, stream);
  else if (lean) (train ? launch_qkv_variant<false, true, true> : launch_qkv_variant<false, false, true>)(a, grid, block, stream);
  else (train ? launch_qkv_variant<false, true, false> : launch_qkv_variant<false, false, false>)(a, grid, block, stream);
  if (fold_apart)
    fold_emb_qkv_mfma(args.fold_wq, args.ld_fold_wq, args.fold_we, args.ld_fold_we, args.fold_out, args.ld_fold_out,
                      args.fold_R, args.fold_d, args.fold_kp, stream);
}

int g_bwd_grid_cap = 0;  // tuning knob (attn_set_bwd_grid); 0 = 256 workgroups per head (measured best)

void launch_bwd_mfma(const AttnArgs& a, hipStream_t stream) {
  // a multiple of Hl workgroups (each owns one head); with the bias gradient,
  // fewer longer-lived workgroups keep its atomics few
  int grid = grid_for(a.B * a.Hl, a.dbias ? (g_bwd_grid_cap > 0 ? g_bwd_grid_cap : 256 * a.Hl) : 4096);
  grid = std::max(a.Hl, grid / a.Hl * a.Hl);
  if (a.D == 32) {
    hipLaunchKernelGGL(k_attn16_bwd<32>, dim3(grid), dim3(256), bwd_lds_bytes<32>(), stream, a);
  } else if (a.D == 64) {
    hipLaunchKernelGGL(k_attn16_bwd<64>, dim3(grid), dim3(256), bwd_lds_bytes<64>(), stream, a);
  } else {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(k_attn16_bwd<128>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)bwd_lds_bytes<128>()) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(k_attn16_bwd<128>, dim3(grid), dim3(256), bwd_lds_bytes<128>(), stream, a);
  }
}

}  // namespace attn
}  // namespace dev
}  // namespace ccmpi
