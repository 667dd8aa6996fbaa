// Large-tile bf16 "NT" GEMM: 8 waves in two ping-pong groups, LDS-DMA
// (global_load_lds) staging with four half-tiles in flight, one MFMA quadrant
// per phase.  Same contract and epilogue as k_gemm_nt (gemm.hip); requires
// K % 128 == 0 (two K-tiles per main-loop iteration).  Two shapes:
//   BN = 256: 256x256 tile, waves 2(M) x 4(N)   (large square-ish problems)
//   BN = 192: 256x192 tile, waves 4(M) x 2(N)   (N = 384 / 768: whole tiles per CU)
//   BN = 128: 256x128 tile, waves 4(M) x 2(N)
//
// Block tile 256(M) x BN(N) x 64(K), 512 threads = 8 waves.
//   * LDS: 2 buffers x {A rows 0-127, A rows 128-255, B rows 0..BN/2-1,
//     B rows BN/2..BN-1} half-tiles (A: 16 KiB, B: BN/2 x 128 B).
//   * Wave (wr, wc) owns rows {mh*128 + wr*(128/WR) + ...} and columns
//     {nh*BN/2 + wc*32 + 0..31} for mh, nh in {0, 1}: every wave reads the
//     SAME half-tiles in the same phase, so a half-tile is free to be restaged
//     as soon as all waves are past its last read.
//   * One K-tile = 4 phases, one (mh, nh) output quadrant (K = 64,
//     v_mfma_f32_16x16x32_bf16) per phase, in the order (0,0) (0,1) (1,1)
//     (1,0).  LDS reads per phase: A0+B0 | B1 | A1 | - (A and B0 fragments
//     stay in registers across phases).
//   * Every phase issues one half-tile of LDS-DMA (1 KiB piece q by wave
//     q % 8) and then waits with vmcnt(2*2 + 2*nB) (nB = this wave's pieces of
//     a B half-tile, 1 or 2): the stage pattern repeats B,A,A,B, so exactly the
//     half-tile issued four phases earlier is retired.  The stage order (below) puts each restage >= 2 phases after its
//     half's last read and each retire >= 1 phase before its first read, which
//     is what the ping-pong barrier pattern requires (analysis in gemm256_schedule
//     comment).
//   * Tile order: XCD-aware remap, then group-M (8 tile rows) so the 32 tiles an
//     XCD runs at once form an 8 x 4 block (A and B panels shared in its L2).
//   * Ping-pong: waves 4-7 execute one extra s_barrier up front, so while one
//     group runs its 16 MFMAs between two barriers the other group issues its
//     LDS reads and DMA; the MFMA cluster runs at s_setprio 1.
//   * Epilogue: the fp32 tile goes through LDS in two 128-row halves and is
//     written with the shared row store (bias / act / bf16 / accumulate /
//     split-K atomics).
//
// gemm256_schedule: let phase p of group 0 sit between barriers #(2p-1) and
// #(2p) and of group 1 between #2p and #(2p+1).  A wave's DMA is visible to a
// reader once the issuing wave waited on it and the reader passed a later
// barrier: retire at phase w -> readable from phase w+1 on.  A restage at
// phase s may overwrite data last read at phase r when s >= r+2.  With
// per-iteration phases P0..P7 (two K-tiles, buffers 0 then 1), the half-tile
// staged at each phase is
//   P0 buf1.B1(t+1) P1 buf1.A1(t+1) P2 buf0.A0(t+2) P3 buf0.B0(t+2)
//   P4 buf0.B1(t+2) P5 buf0.A1(t+2) P6 buf1.A0(t+3) P7 buf1.B0(t+3)
// (t = 2*iteration).  Last reads: buf0 A0,B0@P0 B1@P1 A1@P2; buf1 A0,B0@P4
// B1@P5 A1@P6; first reads one iteration later at the same phases.  Each half
// is staged 2 phases after its last read and retired 4 phases after staging,
// at or before the phase preceding its first read.
#include <hip/hip_runtime.h>

#include "gemm_common.hpp"

namespace ccmpi {
namespace dev {
namespace gemm {
namespace {

constexpr int PM = 256, PK = 64, PNT = 512, kGroupM = 8;
constexpr int kAHalf = 128 * 128;                // bytes per A half-tile

template <int BN>
struct Geo {
  static constexpr int WR = BN == 256 ? 2 : 4;    // wave rows
  static constexpr int WC = 8 / WR;               // wave cols
  static constexpr int MI = 8 / WR;               // 16-row MFMA tiles per wave strip and half
  static constexpr int NS = (BN / 2) / WC;        // wave column strip per B half
  static constexpr int NJ = NS / 16;              // 16-col MFMA tiles per strip
  static constexpr int BHalf = (BN / 2) * 128;    // bytes per B half-tile
  static constexpr int BPieces = BHalf / 1024;    // 1 KiB DMA pieces per B half-tile (piece q -> wave q % 8)
  static constexpr int Buf = 2 * kAHalf + 2 * BHalf;
  static constexpr int EpiTS = BN + 4;
  static constexpr int Lds = (2 * Buf > 128 * EpiTS * 4) ? 2 * Buf : 128 * EpiTS * 4;
  static_assert(NS % 16 == 0 && BPieces >= 8 && BPieces <= 16, "unsupported BN");
};

enum Slot { A0 = 0, A1 = 1, B0 = 2, B1 = 3 };

// TN half-tile image: row r (reduction index) = 256 B = 8 granules of 16 output
// indices; granule g is stored at g ^ tn_swz(r).
__device__ __forceinline__ int tn_swz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int tn_off(int r, int col) {
  return r * 256 + ((((col >> 4) ^ tn_swz(r)) << 5) | ((col & 15) << 1));
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// steady state: this wave's DMA pieces of the last four stages (2 A + 2 B)
__device__ __forceinline__ void wait_steady(int b_pieces) {
  if (b_pieces == 2) wait_vm<8>();
  else wait_vm<6>();
}

// EXP: ablation bits for benchmarks only (0 = production):
//   1 = lax vmcnt (wait for nothing: WRONG results, isolates DMA-latency stalls)
//   2 = no s_setprio around the MFMA cluster
//   4 = no ping-pong stagger (both groups in lockstep)
// TN: weight-gradient form C[N1][N2] = sum_m A[m][n1] B[m][n2] (g.M = N1, g.N = N2,
// g.K = M).  Half-tiles are 64 reduction rows x 128 output indices, stored as
// 256-B rows whose 32-B granules are XOR-swizzled by tn_swz(row); operands come
// out of ds_read_b64_tr_b16 (conflict-free: 16 lanes read rows r..r+3 and, in the
// other lane group, r+8..r+11 -> 8 distinct granules).  Split-K partials go to
// workspace slices (g.C + split * N1 * N2) for k_splitk_reduce.
template <int BN, int EXP = 0, int FAST = 0, bool TN = false>  // FAST: fast_epilogue_id (gemm_common.hpp)
__global__ void __launch_bounds__(PNT, 1) k_gemm_nt_pp(GemmArgs g) {
  using G = Geo<BN>;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + PM - 1) / PM;
  const int nwg = tiles_n * tiles_m * g.splitk;
  int wg = xcd_remap(blockIdx.x, nwg);
  const int split = wg % g.splitk;
  wg /= g.splitk;
  int tm, tn;
  {  // group-M order
    const int per_group = kGroupM * tiles_n;
    const int first_m = (wg / per_group) * kGroupM;
    const int gm = min(tiles_m - first_m, kGroupM);
    tm = first_m + (wg % per_group) % gm;
    tn = (wg % per_group) / gm;
  }
  const int bm = tm * PM, bn = tn * BN;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave / G::WC, wc = wave % G::WC, grp = wave >> 2;

  const int nk_all = g.K / PK;
  const int per = ((nk_all + g.splitk - 1) / g.splitk + 1) & ~1;  // even K-tiles per split
  const int kt0 = split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);             // even (K % 128 == 0)

  auto lds = [&](int buf, int slot) {
    return smem + buf * G::Buf + (slot < 2 ? slot * kAHalf : 2 * kAHalf + (slot - 2) * G::BHalf);
  };

  // DMA of one half-tile in 1 KiB pieces (8 rows x 128 B, one wave instruction).
  // Lane-linear LDS image; the (row & 7) chunk swizzle is applied to the source.
  const int lrow = lane >> 3, pchunk = lane & 7;
  auto stage = [&](int buf, int slot, int kt) {
    if constexpr (TN) {
      // a DMA piece = 4 reduction rows x 256 B; lane -> (row, physical granule, half)
      const bool isA = slot < 2;
      const uint16_t* base = isA ? g.A : g.B;
      const int ld = isA ? g.lda : g.ldb, lim = isA ? g.M : g.N;
      const int r0 = (isA ? bm : bn) + (slot & 1) * 128;
      const int k0 = (kt0 + kt) * PK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = i * 8 + wave;
        const int row = q * 4 + (lane >> 4);
        const int lg = ((lane & 15) >> 1) ^ tn_swz(row);
        int oc = r0 + lg * 16 + (lane & 1) * 8;
        if (oc + 8 > lim) oc = 0;  // outside N1 / N2: any valid address (outputs discarded)
        __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)(k0 + row) * ld + oc),
                                         (__attribute__((address_space(3))) void*)(lds(buf, slot) + q * 1024), 16, 0,
                                         0);
      }
      return;
    }
    const bool isA = slot < 2;
    const uint16_t* base = isA ? g.A : g.B;
    const int ld = isA ? g.lda : g.ldb, lim = (isA ? g.M : g.N) - 1;
    const int r0 = isA ? bm + (slot & 1) * 128 : bn + (slot & 1) * (BN / 2);
    const int k0 = (kt0 + kt) * PK;
    const int npieces = isA ? 16 : G::BPieces;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = i * 8 + wave;
      if (q < npieces) {
        const int r = q * 8 + lrow;
        const int c = pchunk ^ (r & 7);
        const int gr = min(r0 + r, lim);
        __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)gr * ld + k0 + c * 8),
                                         (__attribute__((address_space(3))) void*)(lds(buf, slot) + q * 1024), 16, 0,
                                         0);
      }
    }
  };

  const int b_pieces = (wave + 8 < G::BPieces) ? 2 : 1;  // this wave's share of a B half-tile
  floatx4 acc[2][2][G::MI][G::NJ];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < G::MI; ++i)
#pragma unroll
        for (int j = 0; j < G::NJ; ++j) acc[a][b][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[G::MI][2], fb0[G::NJ][2], fb1[G::NJ][2];
  const int tq = (lane >> 2) & 3, tp = lane & 3, tgrp = lane >> 4;  // ds_read_b64_tr_b16 lane roles
  auto tr8 = [&](const unsigned char* base, int n_loc, int ks) {   // 8 reduction rows of output index n_loc + lane
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef short v8s __attribute__((ext_vector_type(8)));
    const int r = ks * 32 + tgrp * 8 + tq, col = n_loc + 4 * tp;
    const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)(base + tn_off(r, col)));
    const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)(base + tn_off(r + 4, col)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto read_a = [&](int buf, int h) {
    const unsigned char* base = lds(buf, h);
    if constexpr (TN) {
#pragma unroll
      for (int i = 0; i < G::MI; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = tr8(base, wr * (128 / G::WR) + i * 16, ks);
      return;
    }
#pragma unroll
    for (int i = 0; i < G::MI; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int row = wr * (128 / G::WR) + i * 16 + (lane & 15);
        const int chunk = ks * 4 + (lane >> 4);
        fa[i][ks] = *reinterpret_cast<const bf16x8*>(base + row * 128 + ((chunk ^ (row & 7)) << 4));
      }
  };
  auto read_b = [&](int buf, int h, bf16x8 (&fb)[G::NJ][2]) {
    const unsigned char* base = lds(buf, 2 + h);
    if constexpr (TN) {
#pragma unroll
      for (int j = 0; j < G::NJ; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb[j][ks] = tr8(base, wc * G::NS + j * 16, ks);
      return;
    }
#pragma unroll
    for (int j = 0; j < G::NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int row = wc * G::NS + j * 16 + (lane & 15);
        const int chunk = ks * 4 + (lane >> 4);
        fb[j][ks] = *reinterpret_cast<const bf16x8*>(base + row * 128 + ((chunk ^ (row & 7)) << 4));
      }
  };
  auto mma = [&](int mh, int nh, bf16x8 (&fb)[G::NJ][2]) {
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(EXP & 2)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < G::MI; ++i)
#pragma unroll
        for (int j = 0; j < G::NJ; ++j)
          acc[mh][nh][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[j][ks], acc[mh][nh][i][j], 0, 0, 0);
    if constexpr (!(EXP & 2)) __builtin_amdgcn_s_setprio(0);
    bar();
  };
  // retire the half-tile issued four phases ago (steady state) or everything (tail)
  auto retire = [&](bool tail) {
    if constexpr (EXP & 1) {
      if (tail) wait_vm<0>();
    } else {
      if (tail) wait_vm<0>();
      else wait_steady(b_pieces);
    }
  };

  if (nk > 0) {
    // prologue: tile 0 complete in buffer 0, tile 1's A0/B0 in flight
    stage(0, A0, 0);
    stage(0, B0, 0);
    stage(0, B1, 0);
    stage(0, A1, 0);
    stage(1, A0, 1);
    stage(1, B0, 1);
    wait_steady(b_pieces);  // buf0 A0, B0 landed (the 4 younger stages may stay in flight)
  }
  __syncthreads();
  if (!(EXP & 4) && grp == 1) bar();  // group 1 runs one barrier behind group 0

  for (int kt = 0; kt < nk; kt += 2) {
    const bool tail = kt + 2 >= nk;  // no tiles beyond this pair: drain instead of counting
    // ---- K-tile kt (buffer 0)
    read_a(0, 0);
    read_b(0, 0, fb0);
    stage(1, B1, kt + 1);
    retire(tail);
    mma(0, 0, fb0);

    read_b(0, 1, fb1);
    stage(1, A1, kt + 1);
    retire(tail);
    mma(0, 1, fb1);

    read_a(0, 1);
    if (!tail) stage(0, A0, kt + 2);
    retire(tail);
    mma(1, 1, fb1);

    if (!tail) stage(0, B0, kt + 2);
    retire(tail);
    mma(1, 0, fb0);

    // ---- K-tile kt + 1 (buffer 1)
    read_a(1, 0);
    read_b(1, 0, fb0);
    if (!tail) stage(0, B1, kt + 2);
    retire(tail);
    mma(0, 0, fb0);

    read_b(1, 1, fb1);
    if (!tail) stage(0, A1, kt + 2);
    retire(tail);
    mma(0, 1, fb1);

    read_a(1, 1);
    if (kt + 3 < nk) stage(1, A0, kt + 3);
    retire(tail);
    mma(1, 1, fb1);

    if (kt + 3 < nk) stage(1, B0, kt + 3);
    retire(tail);
    mma(1, 0, fb0);
  }
  if (!(EXP & 4) && grp == 0) bar();  // re-align the groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: two passes of 128 rows through LDS
  float* tile = reinterpret_cast<float*>(smem);
  GemmArgs w = g;
  if constexpr (TN) {
    if (g.splitk > 1) {  // this split's partial tile -> its workspace slice
      w.C = reinterpret_cast<float*>(g.C) + (size_t)split * g.M * g.N;
      w.ldc = g.N;
      w.splitk = 1;
    }
  }
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) {
        const int cl = nh * (BN / 2) + wc * G::NS + j * 16 + (lane & 15);
        const float b = load_bias(g, bn + cl, split);
#pragma unroll
        for (int i = 0; i < G::MI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tile[(wr * (128 / G::WR) + i * 16 + (lane >> 4) * 4 + r) * G::EpiTS + cl] =
                (FAST > 0 ? g.alpha * acc[mh][nh][i][j][r] + b : epi(g, acc[mh][nh][i][j][r], b));
      }
    __syncthreads();
    if constexpr (FAST > 0) store_rows_fast<128, BN, PNT, ((FAST - 1) & 1) != 0>(w, tile, G::EpiTS, bm + mh * 128, bn, t);
    else store_rows<128, BN, PNT>(w, tile, G::EpiTS, bm + mh * 128, bn, t);
    __syncthreads();
  }
}

}  // namespace

int gemm256_tiles(int M, int N, int bn) { return ((M + PM - 1) / PM) * ((N + bn - 1) / bn); }

template <int BN, int EXP, int FAST = 0>
static void launch_pp(const GemmArgs& g, hipStream_t stream) {
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_nt_pp<BN, EXP, FAST>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, Geo<BN>::Lds) == hipSuccess;
  }();
  (void)attr;
  const int nwg = gemm256_tiles(g.M, g.N, BN) * g.splitk;
  hipLaunchKernelGGL((k_gemm_nt_pp<BN, EXP, FAST>), dim3(nwg), dim3(PNT), Geo<BN>::Lds, stream, g);
}

// production launches: the common epilogues get branch-free instantiations
template <int BN>
static void launch_pp_prod(const GemmArgs& g, hipStream_t stream) {
  switch (fast_epilogue_id(g)) {
    case 1: return launch_pp<BN, 0, 1>(g, stream);  // fp32 out, no bias
    case 2: return launch_pp<BN, 0, 2>(g, stream);  // bf16 out, no bias
    case 4: return launch_pp<BN, 0, 4>(g, stream);  // bf16 out, fp32 bias
    default: return launch_pp<BN, 0, 0>(g, stream);
  }
}

int g_pp_exp = 0;  // ablation variant (benchmarks only)

void launch_gemm_tn_256(const GemmArgs& g, hipStream_t stream) {
  // partial tiles (split-K) or a plain fp32 tile: branch-free epilogue; accumulate -> generic
  if (g.splitk > 1 || !g.accumulate) {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_nt_pp<256, 0, 1, true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256>::Lds) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL((k_gemm_nt_pp<256, 0, 1, true>), dim3(gemm256_tiles(g.M, g.N, 256) * g.splitk), dim3(PNT),
                       Geo<256>::Lds, stream, g);
  } else {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_nt_pp<256, 0, 0, true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256>::Lds) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL((k_gemm_nt_pp<256, 0, 0, true>), dim3(gemm256_tiles(g.M, g.N, 256) * g.splitk), dim3(PNT),
                       Geo<256>::Lds, stream, g);
  }
}

void launch_gemm_nt_256(const GemmArgs& g, int bn, hipStream_t stream) {
  if (bn == 128) return launch_pp_prod<128>(g, stream);
  if (bn == 192) return launch_pp_prod<192>(g, stream);
  switch (g_pp_exp) {
    case 1: return launch_pp<256, 1>(g, stream);
    case 2: return launch_pp<256, 2>(g, stream);
    case 4: return launch_pp<256, 4>(g, stream);
    case 6: return launch_pp<256, 6>(g, stream);
    default: return launch_pp_prod<256>(g, stream);
  }
}

}  // namespace gemm
}  // namespace dev
}  // namespace ccmpi
