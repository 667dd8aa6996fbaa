// 256x256 bf16 "NT" GEMM with four waves of 128x128 each (one wave per SIMD).
//
// Why this shape (profiles/r3_gemm): hipBLASLt's kernel on the Llama-3-8B MLP
// shapes is MT256x256x64 with four 16x16 MFMA waves (256-thread workgroups, one per
// CU, 130 KB LDS) and keeps the matrix pipe busy 84 % of the time; our 8-wave
// ping-pong kernel (gemm256.hip) gives every wave a 128x64 tile, pays two
// barriers per 16 MFMAs and sits at 54 %.  A 128x128 wave tile halves the LDS
// bytes read per MFMA (16 fragment reads feed 64 MFMAs) and needs one barrier
// per 128 MFMAs.
//
// Per workgroup: C tile 256(M) x 256(N), K-tiles of 64, two LDS stages of
// 64 KiB (A 256 x 128 B + B 256 x 128 B rows, 16-B chunks XOR-swizzled by
// row & 7).  Staging is LDS-DMA (buffer_load ... lds) through one buffer
// descriptor per operand and tile: rows past M / N read as zero (buffer bounds),
// one VGPR of per-lane offset, the K and piece offsets in SGPRs.
//
// Main loop, K-tile t (fragment sets F0 = k 0..31, F1 = k 32..63 of a tile):
//   X: DMA tile t+1 into the other stage | read F0(t)       | 64 MFMA on F1(t-1)
//   Y:                                     read F1(t)       | 64 MFMA on F0(t)
//      vmcnt(0) + lgkmcnt(0) + barrier   (tile t+1 landed; every wave is done
//                                          reading stage t, which the DMA of
//                                          tile t+2 overwrites next)
// so each DMA has two MFMA phases (~2k cycles) to land and each fragment read one.
// Epilogue: per wave, two 64-row halves staged through LDS as fp32, written
// as whole 16-B row vectors (alpha, bias, activation, accumulate, fp32/bf16 out).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <type_traits>

#include "gemm_common.hpp"

namespace ccmpi {
namespace dev {
namespace gemm {
namespace {

constexpr int WM = 256, WNB = 256, WK = 64, WNT = 256;
constexpr int kOpBytes = 256 * 128;           // one operand's K-tile (256 rows x 64 bf16)
constexpr int kStage4 = 2 * kOpBytes;         // A + B
constexpr int kEpiRows = 32;                  // epilogue pass: 32 rows x 128 columns per wave
constexpr int kEpiTS = 132;                   // epilogue fp32 row stride (128 + 4 pad)
constexpr int kEpiWave = kEpiRows * kEpiTS * 4;
// stage 0 | stage 1, the epilogue slabs overlay stage 1 (and a little beyond) so
// a persistent workgroup can prefetch its next tile into stage 0 meanwhile
constexpr int kLds4 = kStage4 + ((kStage4 > 4 * kEpiWave) ? kStage4 : 4 * kEpiWave);

typedef __attribute__((address_space(3))) void* lds_vptr;

constexpr int kLdsExtra = 256;  // after the slabs: fused-epilogue ticket + peers' output pointers

struct W4Args {
  GemmArgs g;
  int group_m;  // tile rows per group of the group-M order
  FusedArgs f;  // FUSED only
  unsigned long long* dbg;  // STAMP diagnostic builds only: 4 cycle counts per wave
  uint16_t* glu;  // EPI 2 only: silu(gate) * up of each interleaved (gate, up) column pair
  int ldglu;
  // EPI 1 push mode (push_rows > 0): output row block j = rows [j * push_rows, (j + 1) *
  // push_rows) goes to push[j] (row 0 of the block at push[j]; a peer's inbox slot), not C
  int push_rows;
  uint16_t* push[kMaxRanks];
  // diagnostic (gemm_set_pair_nobar, wrong results): the pair ring's odd-phase sync reduced to
  // the wave's own waits (1), to the barrier without the DMA wait (2), or to neither (3) --
  // upper bounds of removing the barrier's skew / the DMA latency stalls
  int nobar;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t op_rsrc(const uint16_t* base, long rows, int ld) {
  // rows <= 0: an empty descriptor (every load reads 0)
  long bytes = rows > 0 ? rows * (long)ld * 2 : 0;
  if (bytes > 0x7ffffff0l) bytes = 0x7ffffff0l;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, (int)bytes, 0x00020000);
}

// logical tile -> (tile row, tile column) in group-M order
__device__ __forceinline__ void tile_coords(int wg, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  const int per_group = group_m * tiles_n;
  const int first_m = (wg / per_group) * group_m;
  const int gm = min(tiles_m - first_m, group_m);
  tm = first_m + (wg % per_group) % gm;
  tn = (wg % per_group) / gm;
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return pk_bf16(a, b);
}

// two floats -> packed bf16 (RNE, NaN kept) in one v_cvt_pk_bf16_f32
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  const bf16x2_t h = __builtin_convertvector(float2_t{a, b}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, h);
}

// Fused TP all-reduce epilogue (FusedState comment in gemm_common.hpp).  `to_slab(h)`
// stages this wave's 32-row pass h of the fp32 tile in `tile` (row stride kEpiTS).
template <typename ToSlab>
__device__ void fused_epilogue(const W4Args& wa, int t, int bm, int bn, const float* tile, ToSlab&& to_slab,
                               const float* bias) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const GemmArgs& g = wa.g;
  const FusedArgs& f = wa.f;
  const PeerTable* pt = f.pt;
  const int p = pt->size, me = pt->rank;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wr = wave >> 1, wc = wave & 1;
  const int owner = t % p, lidx = t / p;
  uint32_t* s_ticket = reinterpret_cast<uint32_t*>(smem + kLds4);
  char** s_out = reinterpret_cast<char**>(smem + kLds4 + 64);
  FusedState* own = f.tab->state[me];
  FusedState* ost = f.tab->state[owner];
  uint32_t* err = &pt->sig[me]->error;
  if (threadIdx.x == 0) {
    // publish this call's output (every workgroup writes the same two words), then
    // draw the ticket: the release orders the publication before the ticket
    __hip_atomic_store(&own->out_code[0], f.out_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&own->out_code[1], f.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    release_sys();
    *s_ticket = __hip_atomic_fetch_add(&ost->cnt[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const bool last = *s_ticket == (uint32_t)(p - 1);
  char* inbox = resolve(pt, owner, f.tab->inbox_code[owner]) + (uint64_t)lidx * p * kFusedTileBytes;
  const int cl = (lane & 15) * 8;
  if (!last) {
    // my bf16 partial -> the owner's slot `me` (write-through stores), then flag it
    const Rsrc slot = make_rsrc(uniform_ptr(inbox + (uint64_t)me * kFusedTileBytes), (uint32_t)kFusedTileBytes);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      to_slab(h);
#pragma unroll 2
      for (int it = 0; it < 8; ++it) {
        const int rl = it * 4 + (lane >> 4);
        const float4 x0 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl);
        const float4 x1 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl + 4);
        u32x4 w;
        const float al = g.alpha;
        w[0] = pack_bf16x2(al * x0.x, al * x0.y); w[1] = pack_bf16x2(al * x0.z, al * x0.w);
        w[2] = pack_bf16x2(al * x1.x, al * x1.y); w[3] = pack_bf16x2(al * x1.z, al * x1.w);
        const int row = wr * 128 + h * 32 + rl, col = wc * 128 + cl;
        st16(slot, (uint32_t)((row * 256 + col) * 2), w);
      }
      __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      release_sys();
      signal_store(&ost->ready[t][me], f.seq);
    }
    __syncthreads();  // the slabs are reused by this workgroup's next tile
    return;
  }
  // last arrival: every other rank's partial is (being) stored into the owner's inbox
  bool ok = true;
  if ((int)threadIdx.x < p) {
    const int j = threadIdx.x;
    if (j != me) {
      ok = wait_geq(&ost->ready[t][j], f.seq, f.timeout_ticks, err, 0xA00 + j);
      if (!ok) report_host(pt, 0xA00 + j);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    FusedState* sj = f.tab->state[j];
    const uint64_t code = __hip_atomic_load(&sj->out_code[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t cseq = __hip_atomic_load(&sj->out_code[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (cseq != f.seq) {  // cannot happen when every rank runs the same call sequence
      __hip_atomic_store(err, 0xB00u + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      report_host(pt, 0xB00 + j);
      ok = false;
    }
    s_out[j] = ok ? resolve(pt, j, code) : nullptr;
  }
  ok = __syncthreads_and(ok);
  if (ok) {
    // per pass: this lane's 8 row vectors of 8 columns; the sum runs over the ranks in
    // order (own partial from the slab, the others' from the inbox, 8 loads in flight
    // per rank), then the result is stored into every rank's output
    const uint32_t out_bytes = (uint32_t)min<uint64_t>((uint64_t)g.M * g.ldc * 2, 0x7ffffff0ull);
    for (int h = 0; h < 4; ++h) {
      to_slab(h);
      float v[8][8];
      u32x4 mine[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rl = it * 4 + (lane >> 4);
        const float4 x0 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl);
        const float4 x1 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl + 4);
        const float al = g.alpha;
        mine[it][0] = pack_bf16x2(al * x0.x, al * x0.y); mine[it][1] = pack_bf16x2(al * x0.z, al * x0.w);
        mine[it][2] = pack_bf16x2(al * x1.x, al * x1.y); mine[it][3] = pack_bf16x2(al * x1.z, al * x1.w);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[it][q] = 0.f;
      }
      __builtin_amdgcn_wave_barrier();  // slab reads done before the next pass rewrites it
#pragma unroll 1
      for (int j = 0; j < p; ++j) {
        u32x4 x[8];
        if (j == me) {
#pragma unroll
          for (int it = 0; it < 8; ++it) x[it] = mine[it];
        } else {
          const Rsrc rs = make_rsrc(uniform_ptr(inbox + (uint64_t)j * kFusedTileBytes), (uint32_t)kFusedTileBytes);
#pragma unroll
          for (int it = 0; it < 8; ++it) {
            const int trow = wr * 128 + h * 32 + it * 4 + (lane >> 4), tcol = wc * 128 + cl;
            x[it] = ld16(rs, (uint32_t)((trow * 256 + tcol) * 2));
          }
        }
#pragma unroll
        for (int it = 0; it < 8; ++it)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[it][2 * q] += bf16_lo(x[it][q]);
            v[it][2 * q + 1] += bf16_hi(x[it][q]);
          }
      }
      u32x4 res[8];
#pragma unroll
      for (int it = 0; it < 8; ++it)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          res[it][q] = pack_bf16x2(v[it][2 * q] + bias[2 * q], v[it][2 * q + 1] + bias[2 * q + 1]);
      const int col = bn + wc * 128 + cl;
#pragma unroll 1
      for (int j = 0; j < p; ++j) {
        const Rsrc ro = make_rsrc(uniform_ptr(s_out[j]), out_bytes);
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int row = bm + wr * 128 + h * 32 + it * 4 + (lane >> 4);
          if (row < g.M && col < g.N) st16(ro, (uint32_t)(((uint64_t)row * g.ldc + col) * 2), res[it]);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(&ost->cnt[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // next call's tickets
    release_sys();
    for (int j = 0; j < p; ++j) signal_store(&f.tab->state[j]->done[t], f.seq);
  }
  __syncthreads();
}

// PERSIST: grid = min(tiles, CUs); workgroup b runs logical tiles s, s + G, s + 2G, ...
// (s = XCD-aware remap of b) and prefetches the next tile's first K-tile during the
// epilogue.  ORDER: MFMA-first issue order inside each fenced group.  FRONT: the next
// K-tile's 16 DMA pieces go out in the first half of phase X (4 per group) instead of
// 2 per group over all of it, so each has ~3/4 of a K-tile to land before the barrier.
template <int PERSIST, int ORDER, int FUSED = 0, int FRONT = 0>
__global__ void __launch_bounds__(WNT, 1) k_gemm_w4(W4Args wa) {
  const GemmArgs& g = wa.g;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tiles_n = (g.N + WNB - 1) / WNB, tiles_m = (g.M + WM - 1) / WM;
  const int ntiles = tiles_n * tiles_m;
  const int slot = xcd_remap(blockIdx.x, gridDim.x);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = g.K / WK;

  // ---- staging: 32 pieces of 1 KiB (8 rows x 128 B) per operand and K-tile;
  // wave w issues pieces q = 4 i + w.  Lane l of a piece: row q*8 + (l >> 3),
  // physical chunk l & 7 holding logical chunk (l & 7) ^ (l >> 3).
  const int prow = wave * 8 + (lane >> 3);
  const int pchunk = ((lane & 7) ^ ((lane >> 3) & 7)) << 4;
  const int va = prow * g.lda * 2 + pchunk, vb = prow * g.ldb * 2 + pchunk;
  const int sa = 32 * g.lda * 2, sb = 32 * g.ldb * 2;  // byte step between a wave's pieces
  __amdgpu_buffer_rsrc_t ra, rb;  // the current tile's operand descriptors
  auto ops_for = [&](int tm, int tn) {
    ra = op_rsrc(g.A + (size_t)tm * WM * g.lda, (long)g.M - tm * WM, g.lda);
    rb = op_rsrc(g.B + (size_t)tn * WNB * g.ldb, (long)g.N - tn * WNB, g.ldb);
  };
  auto stage_piece = [&](int buf, int kt, int i) {
    unsigned char* base = smem + buf * kStage4;
    // the piece offsets are recomputed per use (a few SALU ops) instead of 16
    // loop-invariant SGPRs, which pushed the kernel past the SGPR budget (spills)
    int sa_ = sa, sb_ = sb;
    asm volatile("" : "+s"(sa_), "+s"(sb_));
    const int k0 = kt * WK * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_vptr)(base + (i * 4 + wave) * 1024), 16, va, k0 + i * sa_, 0,
                                             0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_vptr)(base + kOpBytes + (i * 4 + wave) * 1024), 16, vb,
                                             k0 + i * sb_, 0, 0);
  };
  auto stage = [&](int buf, int kt) {
#pragma unroll
    for (int i = 0; i < 8; ++i) stage_piece(buf, kt, i);
  };

  // ---- fragments (v_mfma_f32_16x16x32_bf16): lane l holds row (l & 15) of a
  // 16-row block, k = 8 (l >> 4) .. +7 of the 32-deep half `ks`
  const int frow = lane & 15;
  auto rd = [&](int buf, int ks, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const unsigned char* A = smem + buf * kStage4;
    const unsigned char* B = A + kOpBytes;
    const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr * 128 + i * 16 + frow;
      fa[i] = *reinterpret_cast<const bf16x8*>(A + row * 128 + ((chunk ^ (row & 7)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = wc * 128 + j * 16 + frow;
      fb[j] = *reinterpret_cast<const bf16x8*>(B + row * 128 + ((chunk ^ (row & 7)) << 4));
    }
  };
  // group g of a phase reads two fragments of the next set: B blocks 2g, 2g+1 for
  // g < 4, then A blocks 2(g-4), 2(g-4)+1, so the next phase's first MFMAs (A block
  // 0 against every B block) find their operands landed
  auto rd2 = [&](int buf, int ks, int grp, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const unsigned char* base = smem + buf * kStage4 + (grp < 4 ? kOpBytes : 0);
    const int chunk = ks * 4 + (lane >> 4);
    const int b0_ = (grp < 4 ? wc : wr) * 128 + (grp & 3) * 32 + frow;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = b0_ + u * 16;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(base + row * 128 + ((chunk ^ (row & 7)) << 4));
      if (grp < 4) fb[(grp & 3) * 2 + u] = v;
      else fa[(grp & 3) * 2 + u] = v;
    }
  };

  floatx4 acc[8][8];
  auto mma = [&](const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };
  auto sched_y = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
  };
  // inside one fenced group: MFMAs first, each load behind two of them
  auto order_x = [&]() {
    if constexpr (ORDER) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
  auto order_y = [&]() {
    if constexpr (ORDER) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
  };

  const int es = g.out_bf16 ? 2 : 4;
  const bool vec_ok = (((uint64_t)g.C | ((uint64_t)g.ldc * es)) % 16) == 0 && g.N % 8 == 0;
  const int step = PERSIST ? (int)gridDim.x : ntiles;
  int lt = PERSIST ? slot : slot;  // logical tile
  if (lt >= ntiles) return;
  int tm, tn;
  tile_coords(lt, tiles_m, tiles_n, wa.group_m, tm, tn);
  ops_for(tm, tn);
  stage(0, 0);
  for (;;) {
    const int bm = tm * WM, bn = tn * WNB;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a0[8], b0[8], a1[8], b1[8];
    __syncthreads();  // vmcnt(0) + barrier: K-tile 0 landed; the previous epilogue's slab reads are done
    // K-tile 0
    stage(1, min(1, nk - 1));
    rd(0, 0, a0, b0);
    rd(0, 1, a1, b1);
    mma(a0, b0);
    sched_y();
    __syncthreads();
    for (int kt = 1; kt < nk; ++kt) {
      const int buf = kt & 1;
      const int skt = min(kt + 1, nk - 1);  // unconditional: one basic block (last: a harmless re-load)
      // explicit groups: 8 MFMAs + 2 DMA pieces + 2 fragment reads, fenced
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
        if constexpr (FRONT) {
          if (i < 4) {
            stage_piece(buf ^ 1, skt, 2 * i);
            stage_piece(buf ^ 1, skt, 2 * i + 1);
          }
        } else {
          stage_piece(buf ^ 1, skt, i);
        }
        rd2(buf, 0, i, a0, b0);
        if constexpr (!FRONT) order_x();
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
        rd2(buf, 1, i, a1, b1);
        order_y();
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
    }
    // every wave is past its last read of both stages: prefetch the next tile's
    // K-tile 0 into stage 0 while the last MFMAs and the epilogue run
    const int next = lt + step;
    int ntm = 0, ntn = 0;
    if (PERSIST && next < ntiles) {
      tile_coords(next, tiles_m, tiles_n, wa.group_m, ntm, ntn);
      ops_for(ntm, ntn);
      stage(0, 0);
    }
    mma(a1, b1);

    // ---- epilogue: per wave, four 32-row passes through its own slab (over stage 1)
    float* tile = reinterpret_cast<float*>(smem + kStage4 + wave * kEpiWave);
    const int cl = (lane & 15) * 8;
    const int col = bn + wc * 128 + cl;
    float bias[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) bias[q] = load_bias(g, col + q, 0);
    auto to_slab = [&](int h) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tile[(i * 16 + (lane >> 4) * 4 + r) * kEpiTS + j * 16 + (lane & 15)] = acc[h * 2 + i][j][r];
      __builtin_amdgcn_wave_barrier();  // the slab is this wave's own: its LDS accesses run in order
    };
    if constexpr (FUSED) {
      fused_epilogue(wa, tm * tiles_n + tn, bm, bn, tile, to_slab, bias);
    } else {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tile[(i * 16 + (lane >> 4) * 4 + r) * kEpiTS + j * 16 + (lane & 15)] = acc[h * 2 + i][j][r];
      // the slab is this wave's own and a wave's LDS accesses run in order: no barrier
      __builtin_amdgcn_wave_barrier();
#pragma unroll 1
      for (int it = 0; it < 8; ++it) {
        const int rl = it * 4 + (lane >> 4);
        const int row = bm + wr * 128 + h * 32 + rl;
        if (row >= g.M || col >= g.N) continue;
        float v[8];
        const float4 x0 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl);
        const float4 x1 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl + 4);
        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = epi(g, v[q], bias[q]);
        if (vec_ok) {
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
            float* C = reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col;
            float4 y0 = make_float4(v[0], v[1], v[2], v[3]), y1 = make_float4(v[4], v[5], v[6], v[7]);
            if (g.accumulate) {
              const float4 o0 = *reinterpret_cast<const float4*>(C), o1 = *reinterpret_cast<const float4*>(C + 4);
              y0.x += o0.x; y0.y += o0.y; y0.z += o0.z; y0.w += o0.w;
              y1.x += o1.x; y1.y += o1.y; y1.z += o1.z; y1.w += o1.w;
            }
            *reinterpret_cast<float4*>(C) = y0;
            *reinterpret_cast<float4*>(C + 4) = y1;
          }
        } else {
          for (int q = 0; q < 8 && col + q < g.N; ++q) {
            const size_t o = (size_t)row * g.ldc + col + q;
            if (g.out_bf16) {
              uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
              C[o] = (uint16_t)f32_to_bf16_bits(v[q] + (g.accumulate ? bf2f(C[o]) : 0.f));
            } else {
              float* C = reinterpret_cast<float*>(g.C);
              C[o] = v[q] + (g.accumulate ? C[o] : 0.f);
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    }  // !FUSED
    if (!PERSIST || next >= ntiles) break;
    lt = next;
    tm = ntm;
    tn = ntn;
  }
}

// ---------------------------------------------------------------------------------
// Ring kernel (profiles/r3_gemm): the same 256x256 tile and 128x128 wave tiles, but LDS
// is a ring of four 32-KiB slots, each one 32-deep K-step (A 256 x 64 B | B 256 x 64 B).
// A phase is one K-step: 64 MFMAs on the previous step's fragments with the 16 fragment
// reads of this step and the 8 DMA pieces of the step THREE ahead (into the slot read
// two phases ago) hand-interleaved one per MFMA gap, then a counted `s_waitcnt
// vmcnt(16)` (the next step landed, the two after it still in flight) + lgkmcnt(0) +
// a raw s_barrier.
//
// The MFMA takes B's fragment as its A operand (D = B_blk . A_blk^T), so a lane's four
// accumulator values are four CONSECUTIVE output columns of one row: the fast epilogue
// packs them to bf16 (8 B, v_cvt_pk_bf16_f32 + ds_write_b64) into a 32-row slab in slot 3
// and reads back whole 16-B row vectors for the global stores.  PERSIST: grid =
// min(tiles, CUs); after its epilogue a workgroup puts the next tile's first three
// K-steps in flight (slots 0..2) while its stores drain.
//
// In-kernel s_memtime stamps of the previous form (profiles/r3_gemm/stamps.md): 1320-
// 1400 cycles per 1024-MFMA-cycle phase and a 65k-cycle generic epilogue per tile.
//
// 64-B rows: 16-B chunk c of row r sits at physical chunk c ^ f((r >> 2) & 3),
// f = {0, 2, 3, 1}: conflict-free for the 16x16x32 fragment reads (ds_read_b128 lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... each cover the 16 slots of a
// 256-B bank row).  The DMA keeps LDS lane-linear and permutes the source chunk.
constexpr int kRing = 32768;   // one ring slot
constexpr int kRingHalf = 16384;
constexpr int kRingLds = 4 * kRing;
__device__ __forceinline__ int ring_swz(int q) { return (0x78 >> (2 * q)) & 3; }
// pair-slot ring (PAIR): two 64-KiB slots of one 64-deep K pair each (A half, B half:
// 256 rows x 128 B), the fast epilogue's slab (4 x 8 KiB) behind them -- 160 KiB
constexpr int kPair = 65536;
constexpr int kPairHalf = 32768;
constexpr int kPairLds = 2 * kPair + 4 * 8192;

// `younger` vector-memory ops (DMA pieces / epilogue stores) may stay in flight past
// this barrier; every LDS op of the wave has retired
// (every barrier is fenced with sched_barrier(0): the K-major fragment reads are inline
// asm the compiler cannot wait for, so no MFMA may be scheduled above the lgkmcnt(0))
__device__ __forceinline__ void ring_wait_barrier(int younger) {
  __builtin_amdgcn_sched_barrier(0);
  switch (younger) {
    case 63: asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 48: asm volatile("s_waitcnt vmcnt(48) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
  }
  __builtin_amdgcn_sched_barrier(0);
}
template <int YOUNGER>
__device__ __forceinline__ void ring_wait_barrier_c() {
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (YOUNGER == 16) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (YOUNGER == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// one K-step's DMA: slot base + this wave's 1 KiB, per-lane byte offsets incl. the K offset
// (a local struct in the kernel template made hipcc drop the host launch stubs)
struct DmaStep {
  unsigned char* lds;
  int va, vb;    // N layout: every piece; K-major layout: even pieces
  int va1, vb1;  // K-major layout: odd pieces (the swizzle depends on the piece parity)
};

// operand tile descriptor of a K-major ("T") operand stored [K][rows] with row stride ld:
// base at column m0, bounded by the bytes from there to the end of the buffer
__device__ __forceinline__ __amdgpu_buffer_rsrc_t op_rsrc_t(const uint16_t* X, int m0, int K, int ld) {
  long bytes = (long)K * ld * 2 - (long)m0 * 2;
  if (bytes < 0) bytes = 0;
  if (bytes > 0x7ffffff0l) bytes = 0x7ffffff0l;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(X + m0), 0, (int)bytes, 0x00020000);
}

// EPI 1: bf16 out, C = alpha * AB^T, no bias / activation / accumulate (fast epilogue,
// exactly 32 store instructions per wave and tile); EPI 0: the generic epilogue.
// EPI 2: EPI 1 plus the SwiGLU gate of interleaved (gate, up) output column pairs:
// glu[r, c / 2] = silu(C[r, c]) * C[r, c + 1] for even c, from the bf16-rounded C (the
// values the unfused gate would read), one 8-B store next to each 16-B row store.
// ABL (diagnostic ablations, wrong results): bit 2 reads whole 128-B lines per DMA piece
// (8 rows instead of 16 half lines); bit 0 drops the steady-state DMA, bit 1 the
// steady-state fragment reads.  STAMP (diagnostic): per wave, s_memtime cycles of the
// prologue, main loop, epilogue and the phase-end waits -> wa.dbg (first tile only).
// TA / TB: operand layout.  0 ("N"): rows of K contiguous elements (A[m][k], B[n][k]).
// 1 ("T", K-major): stored [K][M] / [K][N] (dX = dY W reads W this way, dW = dY^T X both
// operands).  A K-major slot half is [32 k][256 rows] with 512-B k-rows whose 32-B
// granules are XOR-swizzled by tn_swz(k) (the 256x256 TN kernel's scheme, gemm256.hip);
// its fragments come out of two ds_read_b64_tr_b16 each.
// (Phase placements tried and measured no faster -- reads first / DMA last, odd waves one
// MFMA later, one M0 chain per phase, and for the pair ring front-loaded DMA -- were
// removed; their A/B records: profiles/r4_gemm, profiles/r4_pair2.)
// PAIR (N-layout A; B N-layout or K-major; no diagnostics): the pair-slot ring.  Each DMA piece
// reads 8 whole 128-B lines (8 rows x 64 k) instead of 16 half lines: the 16 x 64-B
// pieces of the 4-slot ring cost 13-16 % against hipBLASLt (profiles/r4_gemm, ABL bit 2
// ablation).  Two slots of one K pair each (kPair): phase q computes step q-1 and reads
// step q from slot (q >> 1) & 1; even phase 2p issues the 16 pieces of pair p+1 into the
// other slot, whose last reader was phase 2p-1; only odd phases end in a barrier (pair
// p+1 landed everywhere, slot p free).
template <int EPI, int PERSIST, int ABL = 0, int STAMP = 0, int TA = 0, int TB = 0, int PAIR = 0>
__global__ void __launch_bounds__(WNT, 1) k_gemm_w4r(W4Args wa) {
  static_assert(!PAIR || (!ABL && !STAMP), "pair-slot ring: no diagnostics");
  const GemmArgs& g = wa.g;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tiles_n = (g.N + WNB - 1) / WNB, tiles_m = (g.M + WM - 1) / WM;
  const int ntiles = tiles_n * tiles_m;
  int lt = xcd_remap(blockIdx.x, gridDim.x);
  if (lt >= ntiles) return;
  const unsigned long long t_start = STAMP ? __builtin_amdgcn_s_memtime() : 0;
  unsigned long long t_wait = 0, t_loop = 0, t_epi = 0;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nst = g.K / 32;
  const int pro = min(nst, 3);  // nst is even: 2 or >= 4
  int tm, tn;
  tile_coords(lt, tiles_m, tiles_n, wa.group_m, tm, tn);
  __amdgpu_buffer_rsrc_t ra, rb;
  auto ops_for = [&](int tm_, int tn_) {
    if constexpr (TA) ra = op_rsrc_t(g.A, tm_ * WM, g.K, g.lda);
    else ra = op_rsrc(g.A + (size_t)tm_ * WM * g.lda, (long)g.M - tm_ * WM, g.lda);
    if constexpr (TB) rb = op_rsrc_t(g.B, tn_ * WNB, g.K, g.ldb);
    else rb = op_rsrc(g.B + (size_t)tn_ * WNB * g.ldb, (long)g.N - tn_ * WNB, g.ldb);
  };
  ops_for(tm, tn);

  // DMA piece i of a step: 16 rows x 64 B; wave w covers rows (4 i + w) * 16 ..
  // lane l: row + (l >> 2), physical chunk l & 3 <- logical chunk (l & 3) ^ f((l >> 4) & 3)
  // (ABL bit 2, diagnostic: each piece reads 8 rows x 128 B -- whole cache lines, as
  // hipBLASLt's 64-deep K tiles do -- instead of 16 rows x 64 B; wrong results)
  const int drow = (ABL & 4) ? wave * 16 + (lane >> 3) : wave * 16 + (lane >> 2);
  const int dchunk = (ABL & 4) ? (lane & 7) << 4 : ((lane & 3) ^ ring_swz((lane >> 4) & 3)) << 4;
  const int va = drow * g.lda * 2 + dchunk, vb = drow * g.ldb * 2 + dchunk;
  // K-major pieces: 2 k-rows x 512 B; wave w, piece i: k-rows 8 i + 2 w + (l >> 5); lane l
  // lands at granule (l & 31) >> 1, half l & 1, holding logical granule ^ tn_swz(k-row)
  const int trow = 2 * wave + (lane >> 5);
  auto vt = [&](int ld, int par) {
    const int sw = (trow & 3) | (par << 2);
    return trow * ld * 2 + (((((lane & 31) >> 1) ^ sw) * 16 + (lane & 1) * 8) * 2);
  };
  const int ta0 = TA ? vt(g.lda, 0) : va, ta1 = TA ? vt(g.lda, 1) : va;
  const int tb0 = TB ? vt(g.ldb, 0) : vb, tb1 = TB ? vt(g.ldb, 1) : vb;
  // piece offsets (N: i * 64 rows, T: i * 8 k-rows): loop-invariant SGPRs (the K offset
  // rides in the VGPR offset, the slot in M0), so a DMA piece costs one M0 write and the load
  const int sa1 = TA ? 16 * g.lda : 64 * g.lda * 2, sb1 = TB ? 16 * g.ldb : 64 * g.ldb * 2;
  const int sa2 = 2 * sa1, sa3 = 3 * sa1, sb2 = 2 * sb1, sb3 = 3 * sb1;
  const int ka = TA ? 64 * g.lda : 64, kb = TB ? 64 * g.ldb : 64;  // bytes per K-step
  auto dma_step = [&](int s) {
    const int sk = (ABL & 4) ? (s >> 1) * 2 : s;  // ABL 4: 128-B aligned K windows
    return DmaStep{smem + (s & 3) * kRing + wave * 1024, ta0 + sk * ka, tb0 + sk * kb, ta1 + sk * ka, tb1 + sk * kb};
  };
  auto dma_piece = [&](const DmaStep& d, int i) {
    const bool isa = i < 4;
    const int so = isa ? (i == 0 ? 0 : i == 1 ? sa1 : i == 2 ? sa2 : sa3)
                       : (i == 4 ? 0 : i == 5 ? sb1 : i == 6 ? sb2 : sb3);
    unsigned char* dst = d.lds + (isa ? 0 : kRingHalf) + (i & 3) * 4096;
    const int vo = isa ? ((TA && (i & 1)) ? d.va1 : d.va) : ((TB && (i & 1)) ? d.vb1 : d.vb);
    if constexpr (TA || TB) {
      // inline asm: hipcc tracks a builtin LDS-DMA as a pending LDS write and puts
      // s_waitcnt vmcnt(0) before every ds_read_b64_tr_b16 (no alias info on the
      // intrinsic), which drained the DMA ring at each transposed read; the ring's
      // counted waits (ring_wait_barrier*) order these loads instead
      const uint32_t m0v = (uint32_t)(uintptr_t)(lds_vptr)dst;
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :
                   : "s"(m0v), "v"(vo), "s"(isa ? ra : rb), "s"(so)
                   : "memory", "m0");
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isa ? ra : rb, (lds_vptr)dst, 16, vo, so, 0, 0);
    }
  };
  auto dma = [&](int s, int i) { dma_piece(dma_step(s), i); };
  // fragment (16x16x32): lane l reads row (l & 15) of a 16-row block, logical chunk l >> 4;
  // the physical chunk depends on the lane only (block rows are multiples of 16)
  const int rdo = (lane & 15) * 64 + (((lane >> 4) ^ ring_swz((lane >> 2) & 3)) << 4);
  // K-major fragment: ds_read_b64_tr_b16 lane roles (group tg = l >> 4 reads k-rows
  // 8 tg + tq (+4), columns 4 tp .. +3 of the 16-row block)
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int tr_base = (tg * 8 + tq) * 512 + tp * 8, tr_swz = tq | ((tg & 1) << 2);
  // inline asm: with the intrinsic, hipcc put s_waitcnt vmcnt(0) before every transposed
  // read (draining the DMA ring).  The compiler does not see these loads complete, so a
  // fragment must only be used after a phase-end barrier (lgkmcnt(0)) -- which is how
  // the ring consumes every fragment -- and the two halves must land in one register
  // tuple without copies (checked in the .s: no v_mov between a read and the barrier)
  auto rd_t = [&](const unsigned char* half, int r0) {
    typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
    const unsigned char* p = half + tr_base + ((((r0 >> 4) ^ tr_swz)) << 5);
    const uint32_t addr = (uint32_t)(uintptr_t)(lds_vptr)p;
    u32x2_t x0, x1;
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:2048"
                 : "=&v"(x0), "=&v"(x1)
                 : "v"(addr));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3));
  };
  // read u (0, 1) of group grp (0..7): B blocks 2 grp + u (grp < 4), then A blocks
  auto rd1 = [&](int s, int grp, int u, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const unsigned char* half = smem + (s & 3) * kRing + (grp < 4 ? kRingHalf : 0);
    const int r0 = (grp < 4 ? wc : wr) * 128 + (grp & 3) * 32 + u * 16;
    const bool t = grp < 4 ? TB : TA;
    const bf16x8 v = t ? rd_t(half, r0) : *reinterpret_cast<const bf16x8*>(half + rdo + r0 * 64);
    if (grp < 4) fb[(grp & 3) * 2 + u] = v;
    else fa[(grp & 3) * 2 + u] = v;
  };

  // ---- PAIR: operand row r at r * 128 B, its 16-B chunk c (k 8 c .. 8 c + 7 of the pair)
  // at physical chunk c ^ ((r >> 1) & 7) -- conflict-free for the fragment reads (each
  // 16-lane ds_read_b128 group: 16 rows, one logical chunk, eight distinct physical ones
  // per row pair).  Piece i (0..7) of an operand, wave w: rows (4 i + w) * 8 .. +7 at LDS
  // i * 4 KiB + w * 1 KiB; lane l -> row + (l >> 3), physical chunk l & 7 <- logical
  // chunk (l & 7) ^ ((w & 1) * 4 + (l >> 4)).
  const int pch = ((lane & 7) ^ (((wave & 1) * 4 + (lane >> 4)) & 7)) << 4;
  const int pva = (wave * 8 + (lane >> 3)) * g.lda * 2 + pch, pvb = (wave * 8 + (lane >> 3)) * g.ldb * 2 + pch;
  const int psa = 32 * g.lda * 2, psb = 32 * g.ldb * 2;  // piece stride: 32 rows
  // PAIR + TB (dX = dY W) / TA (dW = dY^T X, with TB: both operands M-major, no transposes):
  // a K-major operand's half of a pair slot holds the pair's two K-steps in the K-major layout
  // of the 4-slot ring ([32 k][256 rows], 512-B k-rows -- already whole lines), step h at
  // + h * 16 KiB.  Every DMA piece is then inline asm (M0 + load) and the transposed reads use
  // the builtin, which the compiler tracks: with no builtin LDS-DMA in the kernel it adds no
  // vmcnt(0) before them, and no manual lgkmcnt is needed.
  auto dma_asm = [&](unsigned char* dst, __amdgpu_buffer_rsrc_t rs, int vo, int so) {
    const uint32_t m0v = (uint32_t)(uintptr_t)(lds_vptr)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :
                 : "s"(m0v), "v"(vo), "s"(rs), "s"(so)
                 : "memory", "m0");
  };
  auto dma_pair = [&](int p, int i) {  // piece i of pair p: 0..7 A, 8..15 B
    const bool isa = i < 8;
    unsigned char* slot = smem + (p & 1) * kPair;
    if constexpr (TA || TB) {
      // K-major operand: step 2 p + h, piece j of its 16 KiB (the 4-slot ring's layout);
      // an N-layout operand: the pair layout's whole-line pieces
      const int j = i & 3, h = (i & 7) >> 2;
      if (isa) {
        if constexpr (TA)
          dma_asm(slot + h * 16384 + j * 4096 + wave * 1024, ra, ((j & 1) ? ta1 : ta0) + (2 * p + h) * ka,
                  j == 0 ? 0 : j == 1 ? sa1 : j == 2 ? sa2 : sa3);
        else
          dma_asm(slot + (i & 7) * 4096 + wave * 1024, ra, pva + p * 128, (i & 7) * psa);
      } else {
        if constexpr (TB)
          dma_asm(slot + kPairHalf + h * 16384 + j * 4096 + wave * 1024, rb, ((j & 1) ? tb1 : tb0) + (2 * p + h) * kb,
                  j == 0 ? 0 : j == 1 ? sb1 : j == 2 ? sb2 : sb3);
        else
          dma_asm(slot + kPairHalf + (i & 7) * 4096 + wave * 1024, rb, pvb + p * 128, (i & 7) * psb);
      }
    } else {
      unsigned char* dst = slot + (isa ? 0 : kPairHalf) + (i & 7) * 4096 + wave * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isa ? ra : rb, (lds_vptr)dst, 16, (isa ? pva : pvb) + p * 128,
                                               (i & 7) * (isa ? psa : psb), 0, 0);
    }
  };
  // fragment of K-step h (0, 1) of a pair: row (l & 15), logical chunk 4 h + (l >> 4)
  const int prd0 = (lane & 15) * 128 + (((lane >> 4) ^ ((lane & 15) >> 1)) << 4);
  const int prd1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ ((lane & 15) >> 1)) << 4);
  auto rd_tb = [&](const unsigned char* half, int r0) {
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4s* lds_v4s;
    const unsigned char* p = half + tr_base + ((((r0 >> 4) ^ tr_swz)) << 5);
    const v4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s)(lds_vptr)p);
    const v4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s)(lds_vptr)(p + 2048));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto rd_pair = [&](const unsigned char* slot, int h, int grp, int u, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const int r0 = (grp < 4 ? wc : wr) * 128 + (grp & 3) * 32 + u * 16;
    bf16x8 v;
    if (TB && grp < 4) v = rd_tb(slot + kPairHalf + h * 16384, r0);
    else if (TA && grp >= 4) v = rd_tb(slot + h * 16384, r0);  // K-major A (dW = dY^T X): same fragment layout
    else v = *reinterpret_cast<const bf16x8*>(slot + (grp < 4 ? kPairHalf : 0) + (h ? prd1 : prd0) + r0 * 128);
    if (grp < 4) fb[(grp & 3) * 2 + u] = v;
    else fa[(grp & 3) * 2 + u] = v;
  };

  floatx4 acc[8][8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  // acc[i][j] (A block i, B block j): lane l holds C[16 i + (l & 15)][16 j + 4 (l >> 4) + r]
  auto mfma = [&](int i, int j, const bf16x8& fa, const bf16x8& fb) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa, acc[i][j], 0, 0, 0);
  };

  // one phase: MFMAs on (pa, pb) = step q-1, reads of step q into (ca, cb), DMA of step
  // q+3 (DMA), one non-MFMA op per gap: MFMA | read | 2 MFMA | DMA | 2 MFMA | read | 3 MFMA
  auto phase = [&](auto dma_c, auto younger_c, int q, const bf16x8 (&pa)[8], const bf16x8 (&pb)[8],
                   bf16x8 (&ca)[8], bf16x8 (&cb)[8]) {
    constexpr bool DMA = decltype(dma_c)::value;
    constexpr int YOUNGER = decltype(younger_c)::value;
    const DmaStep ds = dma_step(q + 3);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      auto mm = [&](int j0, int j1) {
#pragma unroll
        for (int j = j0; j < j1; ++j) mfma(i, j, pa[i], pb[j]);
        __builtin_amdgcn_sched_barrier(0);
      };
      if constexpr (TA || TB) {
        // K-major operands need ~16 more VGPRs of read offsets: A fragments are
        // replaced in place (pa == ca), block i read right after its last MFMA
        mm(0, 1);
        if constexpr (!(ABL & 2)) rd1(q, i >> 1, i & 1, ca, cb);  // B block i
        __builtin_amdgcn_sched_barrier(0);
        mm(1, 3);
        if constexpr (DMA && !(ABL & 1)) dma_piece(ds, i);
        __builtin_amdgcn_sched_barrier(0);
        mm(3, 8);
        if constexpr (!(ABL & 2)) rd1(q, 4 + (i >> 1), i & 1, ca, cb);  // A block i
        __builtin_amdgcn_sched_barrier(0);
      } else {
        mm(0, 1);
        if constexpr (!(ABL & 2)) rd1(q, i, 0, ca, cb);
        __builtin_amdgcn_sched_barrier(0);
        mm(1, 3);
        if constexpr (DMA && !(ABL & 1)) dma_piece(ds, i);
        __builtin_amdgcn_sched_barrier(0);
        mm(3, 5);
        if constexpr (!(ABL & 2)) rd1(q, i, 1, ca, cb);
        __builtin_amdgcn_sched_barrier(0);
        mm(5, 8);
      }
    }
    if constexpr (STAMP) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      ring_wait_barrier_c<YOUNGER>();
      t_wait += __builtin_amdgcn_s_memtime() - t0;
    } else {
      ring_wait_barrier_c<YOUNGER>();
    }
  };
  using T = std::true_type;
  using F = std::false_type;
  using Y16 = std::integral_constant<int, 16>;
  using Y8 = std::integral_constant<int, 8>;
  using Y0 = std::integral_constant<int, 0>;

  // PAIR phase q: MFMAs on (pa, pb) = step q-1, reads of step q into (ca, cb); even phases
  // with DMA also issue the 16 pieces of pair (q >> 1) + 1, odd phases end in the barrier.
  // Per 8 MFMAs: MFMA | DMA | read | 2 MFMA | DMA | 2 MFMA | read | 3 MFMA
  auto phase_pair = [&](auto dma_c, auto odd_c, int q, const bf16x8 (&pa)[8], const bf16x8 (&pb)[8],
                        bf16x8 (&ca)[8], bf16x8 (&cb)[8]) {
    constexpr bool DMA = decltype(dma_c)::value, ODD = decltype(odd_c)::value;
    const unsigned char* slot = smem + ((q >> 1) & 1) * kPair;
    const int ro = ODD ? 1 : 0;  // K-step within the pair
    const int np = (q >> 1) + 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      auto mm = [&](int j0, int j1) {
#pragma unroll
        for (int j = j0; j < j1; ++j) mfma(i, j, pa[i], pb[j]);
        __builtin_amdgcn_sched_barrier(0);
      };
      mm(0, 1);
      if constexpr (DMA) dma_pair(np, 2 * i);
      rd_pair(slot, ro, i, 0, ca, cb);
      __builtin_amdgcn_sched_barrier(0);
      mm(1, 3);
      if constexpr (DMA) dma_pair(np, 2 * i + 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(3, 5);
      rd_pair(slot, ro, i, 1, ca, cb);
      __builtin_amdgcn_sched_barrier(0);
      mm(5, 8);
    }
    if constexpr (ODD) {
      if (wa.nobar == 1) {  // own waits only, no barrier
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      } else if (wa.nobar == 2) {  // barrier, DMA not waited for
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      } else if (wa.nobar == 3) {  // neither
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      } else {
        ring_wait_barrier_c<0>();
      }
    }
  };

  const int ldc = g.ldc;
  // prologue of the first tile: steps 0..2 in flight (PAIR: pairs 0 and 1)
  auto prologue = [&]() {
    if constexpr (PAIR) {
#pragma unroll
      for (int i = 0; i < 16; ++i) dma_pair(0, i);
      if (nst >= 4)
#pragma unroll
        for (int i = 0; i < 16; ++i) dma_pair(1, i);
    } else {
      for (int s = 0; s < pro; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) dma(s, i);
    }
  };
  prologue();
  // DMA pieces issued after step 0's (PAIR: after pair 0's)
  const int younger0 = PAIR ? (nst >= 4 ? 16 : 0) : 8 * (pro - 1);
  int younger = younger0;
  for (;;) {
    const int bm = tm * WM, bn = tn * WNB;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int next = lt + (int)gridDim.x;
    bool more = false;
    int ntm = 0, ntn = 0;
    if constexpr (PAIR) {
      const int npair = nst >> 1;
      // pair 0 landed everywhere, every wave past the previous tile's epilogue
      ring_wait_barrier(younger);
      // "phase 0": step 0's fragments; phase 1 ends with pair 1 landed
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        rd_pair(smem, 0, i, 0, a0, b0);
        rd_pair(smem, 0, i, 1, a0, b0);
      }
      phase_pair(F{}, T{}, 1, a0, b0, a1, b1);
      for (int p = 1; p + 1 < npair; ++p) {
        phase_pair(T{}, F{}, 2 * p, a1, b1, a0, b0);
        phase_pair(F{}, T{}, 2 * p + 1, a0, b0, a1, b1);
      }
      if (npair > 1) {
        phase_pair(F{}, F{}, nst - 2, a1, b1, a0, b0);
        phase_pair(F{}, T{}, nst - 1, a0, b0, a1, b1);
      }
      // persistent: both slots are free (the last phase's barrier) -- the next tile's
      // pairs 0 and 1 load under the last MFMAs and the epilogue (whose slab is apart)
      more = PERSIST && (EPI == 1 || EPI == 2) && next < ntiles;
      if (more) {
        tile_coords(next, tiles_m, tiles_n, wa.group_m, ntm, ntn);
        ops_for(ntm, ntn);
        prologue();
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) mfma(i, j, a1[i], b1[j]);
    } else {
    // step 0 landed everywhere (and every wave is done with the previous epilogue's slab);
    // "phase 0": step 0's fragments read, step 3 into slot 3, step 1 landed
    ring_wait_barrier(younger);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      rd1(0, i, 0, a0, b0);
      rd1(0, i, 1, a0, b0);
      if (nst >= 4) dma(3, i);
    }
    ring_wait_barrier(nst >= 4 ? 16 : 0);
    if (STAMP) t_loop = __builtin_amdgcn_s_memtime();
    // steady state: phases 1 .. nst-4 in pairs, each prefetching the step three ahead
    // (K-major variants: one A set, a1 aliases a0)
    bf16x8 (&a1r)[8] = (TA || TB) ? a0 : a1;
    for (int q = 1; q + 3 < nst; q += 2) {
      phase(T{}, Y16{}, q, a0, b0, a1r, b1);
      phase(T{}, Y16{}, q + 1, a1r, b1, a0, b0);
    }
    if (nst >= 4) {  // drain: phases nst-3, nst-2, nst-1
      phase(F{}, Y8{}, nst - 3, a0, b0, a1r, b1);
      phase(F{}, Y0{}, nst - 2, a1r, b1, a0, b0);
    }
    phase(F{}, Y0{}, nst - 1, a0, b0, a1r, b1);
    // persistent, fast epilogue: every wave is past its last fragment read (the last
    // phase's barrier), so slots 0..2 are free -- the next tile's first three steps load
    // into them under the last MFMAs and the epilogue (which uses slot 3 only)
    more = PERSIST && (EPI == 1 || EPI == 2) && next < ntiles;
    if (more) {
      tile_coords(next, tiles_m, tiles_n, wa.group_m, ntm, ntn);
      ops_for(ntm, ntn);
      for (int s = 0; s < pro; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) dma(s, i);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma(i, j, a1r[i], b1[j]);
    }
    if (STAMP) t_epi = __builtin_amdgcn_s_memtime();

    if constexpr (EPI == 1 || EPI == 2) {
      // ---- fast epilogue: per 32-row pass, bf16 pairs -> slab (slot 3, 8 KiB per wave,
      // 16-B chunk c of row r at c ^ (r & 15)) -> 16-B row vectors -> buffer stores
      // (PAIR: the slab behind the two pair slots)
      unsigned char* slab = smem + (PAIR ? 2 * kPair : 3 * kRing) + wave * 8192;
      const int grp = lane >> 4, lr = lane & 15;
      const float al = g.alpha;
      const int ccol = bn + wc * 128 + lr * 8;
      uint16_t* cbase = reinterpret_cast<uint16_t*>(g.C);
      int crow = bm + wr * 128;
      if (EPI == 1 && wa.push_rows) {  // whole tiles per block (push_rows % 256 == 0)
        const int blk = bm / wa.push_rows;
        cbase = wa.push[blk];
        crow -= blk * wa.push_rows;
      }
      uint16_t* cptr = cbase + (size_t)crow * ldc + ccol;
      // push mode: the rows go to a peer's inbox over xGMI -- stored write-through (sc0 sc1,
      // kStorePolicy) like every collective store, through a descriptor on the wave-uniform
      // row base, so they leave this XCD's L2 as they are produced and the inbox-to-local
      // collective that follows never depends on an L2 write-back
      const bool pushed = EPI == 1 && wa.push_rows;
      const Rsrc prs = make_rsrc(uniform_ptr(reinterpret_cast<char*>(cbase + (size_t)crow * ldc)), 0x7ffffff0u);
      const int rows_left = g.M - bm - wr * 128;
      const bool col_ok = ccol < g.N;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const floatx4 v = acc[2 * h + ii][j];
            const uint32_t lo = cvt_pk_bf16(al * v[0], al * v[1]);
            const uint32_t hi = cvt_pk_bf16(al * v[2], al * v[3]);
            const int row = ii * 16 + lr, chunk = 2 * j + (grp >> 1);
            *reinterpret_cast<uint2*>(slab + row * 256 + ((chunk ^ (row & 15)) << 4) + (grp & 1) * 8) =
                uint2{lo, hi};
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int rl = it * 4 + grp;
          const u32x4 w = *reinterpret_cast<const u32x4*>(slab + rl * 256 + ((lr ^ (rl & 15)) << 4));
          if (col_ok && h * 32 + rl < rows_left) {
            if (pushed)
              __builtin_amdgcn_raw_buffer_store_b128(w, prs.r, (uint32_t)(((h * 32 + rl) * ldc + ccol) * 2), 0,
                                                     kStorePolicy);
            else
              *reinterpret_cast<u32x4*>(cptr + (size_t)(h * 32 + rl) * ldc) = w;
            if constexpr (EPI == 2) {
              float gl[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float gv = __uint_as_float(w[q] << 16), uv = __uint_as_float(w[q] & 0xffff0000u);
                gl[q] = gv * __builtin_amdgcn_rcpf(1.0f + __expf(-gv)) * uv;
              }
              uint16_t* gp = wa.glu + (size_t)(bm + wr * 128 + h * 32 + rl) * wa.ldglu + (ccol >> 1);
              *reinterpret_cast<uint2*>(gp) = uint2{cvt_pk_bf16(gl[0], gl[1]), cvt_pk_bf16(gl[2], gl[3])};
            }
          }
        }
      }
    } else {
      // ---- generic epilogue (alpha, bias, activation, accumulate, fp32 / bf16 out):
      // per 32-row pass, fp32 through a slab over slots 0..2, one row vector per lane
      float* tile = reinterpret_cast<float*>(smem + wave * kEpiWave);
      const int cl = (lane & 15) * 8;
      const int col = bn + wc * 128 + cl;
      float bias[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) bias[q] = load_bias(g, col + q, 0);
      const int es = g.out_bf16 ? 2 : 4;
      const bool vec_ok = (((uint64_t)g.C | ((uint64_t)ldc * es)) % 16) == 0 && g.N % 8 == 0;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              tile[(i * 16 + (lane & 15)) * kEpiTS + j * 16 + (lane >> 4) * 4 + r] = acc[h * 2 + i][j][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int it = 0; it < 8; ++it) {
          const int rl = it * 4 + (lane >> 4);
          const int row = bm + wr * 128 + h * 32 + rl;
          if (row >= g.M || col >= g.N) continue;
          float v[8];
          const float4 x0 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl);
          const float4 x1 = *reinterpret_cast<const float4*>(tile + rl * kEpiTS + cl + 4);
          v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = epi(g, v[q], bias[q]);
          if (vec_ok) {
            if (g.out_bf16) {
              uint16_t* C = reinterpret_cast<uint16_t*>(g.C) + (size_t)row * ldc + col;
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
              float* C = reinterpret_cast<float*>(g.C) + (size_t)row * ldc + col;
              float4 y0 = make_float4(v[0], v[1], v[2], v[3]), y1 = make_float4(v[4], v[5], v[6], v[7]);
              if (g.accumulate) {
                const float4 o0 = *reinterpret_cast<const float4*>(C), o1 = *reinterpret_cast<const float4*>(C + 4);
                y0.x += o0.x; y0.y += o0.y; y0.z += o0.z; y0.w += o0.w;
                y1.x += o1.x; y1.y += o1.y; y1.z += o1.z; y1.w += o1.w;
              }
              *reinterpret_cast<float4*>(C) = y0;
              *reinterpret_cast<float4*>(C + 4) = y1;
            }
          } else {
            for (int q = 0; q < 8 && col + q < g.N; ++q) {
              const size_t o = (size_t)row * ldc + col + q;
              if (g.out_bf16) {
                uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
                C[o] = (uint16_t)f32_to_bf16_bits(v[q] + (g.accumulate ? bf2f(C[o]) : 0.f));
              } else {
                float* C = reinterpret_cast<float*>(g.C);
                C[o] = v[q] + (g.accumulate ? C[o] : 0.f);
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    // the next tile's top-of-tile wait for its step 0: the epilogue's global stores are
    // younger than the prefetched steps; an interior tile issued exactly 32 (EPI 1) or 64
    // (EPI 2, + the gate) per wave, so they may stay in flight (vmcnt counts at most 63:
    // EPI 2 then also waits for steps 1-2); an edge tile skips some (masked-off waves),
    // then the wait conservatively also retires the stores
    if (more) {
      const bool interior = bm + WM <= g.M && bn + WNB <= g.N;
      younger = !interior ? younger0 : (EPI == 2 ? 63 : younger0 + 32);
    }
    if constexpr (STAMP) {
      if (lt == xcd_remap(blockIdx.x, gridDim.x)) {  // first tile of this workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
          unsigned long long* d = wa.dbg + ((size_t)blockIdx.x * 4 + wave) * 4;
          d[0] = t_loop - t_start;
          d[1] = t_epi - t_loop;
          d[2] = t_end - t_epi;
          d[3] = t_wait;
        }
      }
    }
    if (!more) break;
    lt = next;
    tm = ntm;
    tn = ntn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

int g_w4_sched = 1;   // bit 0: persistent grid, bit 1: MFMA-first order inside groups, bit 2: front-loaded DMA,
                      // bit 3: LDS-ring kernel (k_gemm_w4r), bits 5-6 / 9: its ablations / stamps
int g_w4_group_m = 8;
unsigned long long* g_w4_dbg = nullptr;
long long g_ring_launches = 0;
// auto dispatch: the pair-slot ring (0.93-0.95x hipBLASLt on the Llama MLP shapes against
// 0.86-0.89x for the 4-slot ring, profiles/r4_pair); CCMPI_RING_SCHED overrides (A/B runs)
// K-major A on the pair ring without K-major B (CCMPI_PAIR_TA=1): the TA + TB form is the
// default for dW = dY^T X; A alone goes to the 4-slot ring unless asked for
int g_pair_nobar = 0;
int g_pair_ta = std::getenv("CCMPI_PAIR_TA") ? std::atoi(std::getenv("CCMPI_PAIR_TA")) : 0;
int g_ring_sched = std::getenv("CCMPI_RING_SCHED") ? std::atoi(std::getenv("CCMPI_RING_SCHED")) : (8 | 16384);
long long g_ring_min_macs = std::getenv("CCMPI_RING_MIN_MACS") ? std::atoll(std::getenv("CCMPI_RING_MIN_MACS")) : (1ll << 33);

bool gemm_w4_ok(const GemmArgs& g) {
  // one descriptor per operand tile: the bytes from a tile's first row must fit 2 GiB
  return g.splitk == 1 && g.K % WK == 0 && g.K >= WK && g.lda % 8 == 0 && g.ldb % 8 == 0 &&
         (long)g.M * g.lda * 2 < 0x7ffffff0l && (long)g.N * g.ldb * 2 < 0x7ffffff0l;
}

// After the fused GEMM: this rank's output is final once every tile's reducer has
// flagged it (bounded spins; a timeout records 0xC00 and the kernel returns).
__global__ void __launch_bounds__(256) k_fused_wait(FusedArgs f, int tiles) {
  const PeerTable* pt = f.pt;
  const int me = pt->rank;
  FusedState* own = f.tab->state[me];
  bool ok = true;
  for (int t = threadIdx.x; t < tiles && ok; t += blockDim.x) {
    ok = wait_geq(&own->done[t], f.seq, f.timeout_ticks, &pt->sig[me]->error, 0xC00);
    if (!ok) report_host(pt, 0xC00);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

static void w4_attr(const void* f) {
  (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLds4 + kLdsExtra);
}

// four-slot LDS ring kernel: EPI 1 (fast) when the output is bf16 with no bias, activation
// or accumulation and C rows are 16-B vectors; persistent grid (g_w4_sched bit 0) then.
// Diagnostics: sched bits 5-6 ablations, bit 9 s_memtime stamps (g_w4_dbg).
static void w4r_attr(const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kRingLds); }
static void w4p_attr(const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kPairLds); }

bool gemm_w4r_fast(const GemmArgs& g) {
  return g.out_bf16 && !g.accumulate && g.act == 0 && g.bias_kind == 0 && g.splitk == 1 && g.N % 8 == 0 && g.ldc % 8 == 0 &&
         ((uint64_t)g.C % 16) == 0 && (uint64_t)g.M * g.ldc * 2 < 0x7ffffff0ull;
}

void launch_gemm_nt_w4r(const GemmArgs& g, hipStream_t stream) { launch_gemm_ring(g, 0, 0, stream); }

bool gemm_ring_ok(const GemmArgs& g, int ta, int tb) {
  if (g.splitk != 1 || g.K % WK || g.K < WK || g.lda % 8 || g.ldb % 8 || ((uint64_t)g.A % 16) || ((uint64_t)g.B % 16))
    return false;
  const long a_bytes = ta ? (long)g.K * g.lda * 2 : (long)g.M * g.lda * 2;
  const long b_bytes = tb ? (long)g.K * g.ldb * 2 : (long)g.N * g.ldb * 2;
  // (a K-major operand's byte offsets, K * ld * 2 at most, are 32-bit buffer offsets)
  return a_bytes < 0x7ffffff0l && b_bytes < 0x7ffffff0l;
}

void launch_gemm_ring(const GemmArgs& g, int ta, int tb, hipStream_t stream, uint16_t* glu, int ldglu,
                      uint16_t* const* push, int push_rows) {
  // explicit ring schedule (gemm_set_kernel(5) + sched bit 3) or the auto defaults
  const int sched = (g_w4_sched & 8) ? g_w4_sched : g_ring_sched;
  ++g_ring_launches;
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }();
  static bool attr = [] {
    // 4-slot ring: generic / fast / persistent / SwiGLU epilogues, diagnostics, K-major forms
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<2, 0>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 2>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 3>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 4>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 1, 0, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 0, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 0, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 1, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 1, 1>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 1, 0>));
    w4r_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 1, 0>));
    // pair-slot ring
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 0, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 0, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<2, 0, 0, 0, 0, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 1, 0, 0, 0, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<2, 1, 0, 0, 0, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 0, 1, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 0, 1, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 1, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 1, 0, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<0, 0, 0, 0, 1, 1, 1>));
    w4p_attr(reinterpret_cast<const void*>(k_gemm_w4r<1, 0, 0, 0, 1, 1, 1>));
    return true;
  }();
  (void)attr;
  const int ntiles = gemm_w4_tiles(g.M, g.N);
  W4Args a{g, g_w4_group_m, {}, g_w4_dbg, glu, ldglu};
  a.nobar = g_pair_nobar;
  const bool fast = gemm_w4r_fast(g);
  if (push_rows) {  // row blocks into peers' inboxes: the fast NT epilogue, whole tiles per block
    const int blocks = push_rows > 0 ? g.M / push_rows : 0;
    if (!fast || ta || tb || glu || push_rows % 256 || blocks < 1 || blocks > kMaxRanks || blocks * push_rows != g.M)
      throw std::invalid_argument("gemm ring: push mode needs the fast NT form and M = blocks x push_rows (% 256)");
    a.push_rows = push_rows;
    for (int j = 0; j < blocks; ++j) a.push[j] = push[j];
  }
  const bool pair = sched & 16384;
  const bool persist = fast && (sched & 1);
  const int grid = persist ? std::min(ntiles, cus) : ntiles;
  if (glu) {  // SwiGLU epilogue (callers check gemm_w4r_fast and the glu layout first)
    if (!fast || ta || tb) throw std::invalid_argument("gemm ring: the SwiGLU epilogue needs the fast NT form");
    if (pair && persist) hipLaunchKernelGGL((k_gemm_w4r<2, 1, 0, 0, 0, 0, 1>), dim3(grid), dim3(WNT), kPairLds, stream, a);
    else if (pair) hipLaunchKernelGGL((k_gemm_w4r<2, 0, 0, 0, 0, 0, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a);
    else hipLaunchKernelGGL((k_gemm_w4r<2, 0>), dim3(ntiles), dim3(WNT), kRingLds, stream, a);
    return;
  }
  if ((ta || tb) && pair && (tb || g_pair_ta)) {
    // K-major operands on the pair-slot ring: dX = dY W (B), dW = dY^T X (A and B: no
    // transposes); K-major A alone only on request (CCMPI_PAIR_TA)
    const int v = (ta ? 2 : 0) + (tb ? 1 : 0) + (fast ? 4 : 0);
    switch (v) {
      case 1: hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 0, 1, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a); break;
      case 5: hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 0, 1, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a); break;
      case 2: hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 1, 0, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a); break;
      case 6: hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 1, 0, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a); break;
      case 3: hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 1, 1, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a); break;
      default: hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 1, 1, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a); break;
    }
    return;
  }
  if (ta || tb) {  // K-major operands on the 4-slot ring: non-persistent, no diagnostics
    const int v = (ta ? 2 : 0) + (tb ? 1 : 0) + (fast ? 4 : 0);
    switch (v) {
      case 1: hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 0, 1>), dim3(ntiles), dim3(WNT), kRingLds, stream, a); break;
      case 5: hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 0, 1>), dim3(ntiles), dim3(WNT), kRingLds, stream, a); break;
      case 2: hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 1, 0>), dim3(ntiles), dim3(WNT), kRingLds, stream, a); break;
      case 6: hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 1, 0>), dim3(ntiles), dim3(WNT), kRingLds, stream, a); break;
      case 3: hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 1, 1>), dim3(ntiles), dim3(WNT), kRingLds, stream, a); break;
      default: hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 1, 1>), dim3(ntiles), dim3(WNT), kRingLds, stream, a); break;
    }
    return;
  }
  const int abl = (sched >> 5) & 3;
  if (pair) {
    // pair-slot ring: whole-line DMA pieces, 64-deep slots (bit 0: persistent grid)
    if (persist) hipLaunchKernelGGL((k_gemm_w4r<1, 1, 0, 0, 0, 0, 1>), dim3(grid), dim3(WNT), kPairLds, stream, a);
    else if (fast) hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 0, 0, 0, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a);
    else hipLaunchKernelGGL((k_gemm_w4r<0, 0, 0, 0, 0, 0, 1>), dim3(ntiles), dim3(WNT), kPairLds, stream, a);
  } else if (!fast) {
    hipLaunchKernelGGL((k_gemm_w4r<0, 0>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else if (sched & 512) {  // diagnostic: s_memtime stamps
    if (persist) hipLaunchKernelGGL((k_gemm_w4r<1, 1, 0, 1>), dim3(grid), dim3(WNT), kRingLds, stream, a);
    else hipLaunchKernelGGL((k_gemm_w4r<1, 0, 0, 1>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else if (sched & 8192) {
    // diagnostic: whole-cache-line DMA pieces (ABL 4, wrong results)
    hipLaunchKernelGGL((k_gemm_w4r<1, 0, 4>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else if (abl == 1) {
    hipLaunchKernelGGL((k_gemm_w4r<1, 0, 1>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else if (abl == 2) {
    hipLaunchKernelGGL((k_gemm_w4r<1, 0, 2>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else if (abl == 3) {
    hipLaunchKernelGGL((k_gemm_w4r<1, 0, 3>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else if (persist) {
    hipLaunchKernelGGL((k_gemm_w4r<1, 1>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  } else {
    hipLaunchKernelGGL((k_gemm_w4r<1, 0>), dim3(grid), dim3(WNT), kRingLds, stream, a);
  }
}

void launch_gemm_nt_w4(const GemmArgs& g, hipStream_t stream) {
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }();
  const int ntiles = ((g.M + WM - 1) / WM) * ((g.N + WNB - 1) / WNB);
  W4Args a{g, g_w4_group_m, {}, nullptr};
  const bool persist = g_w4_sched & 1;
  const int grid = persist ? std::min(ntiles, cus) : ntiles;
  static bool attr = [] {
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<0, 0>));
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<1, 0>));
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<0, 1>));
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<1, 1>));
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<0, 0, 0, 1>));
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<1, 0, 0, 1>));
    return true;
  }();
  (void)attr;
  if (g_w4_sched & 8) {
    launch_gemm_nt_w4r(g, stream);
    return;
  }
  if (g_w4_sched & 4) {
    if (persist) hipLaunchKernelGGL((k_gemm_w4<1, 0, 0, 1>), dim3(grid), dim3(WNT), kLds4 + kLdsExtra, stream, a);
    else hipLaunchKernelGGL((k_gemm_w4<0, 0, 0, 1>), dim3(grid), dim3(WNT), kLds4 + kLdsExtra, stream, a);
    return;
  }
  switch (g_w4_sched & 3) {
    case 0: hipLaunchKernelGGL((k_gemm_w4<0, 0>), dim3(grid), dim3(WNT), kLds4 + kLdsExtra, stream, a); break;
    case 1: hipLaunchKernelGGL((k_gemm_w4<1, 0>), dim3(grid), dim3(WNT), kLds4 + kLdsExtra, stream, a); break;
    case 2: hipLaunchKernelGGL((k_gemm_w4<0, 1>), dim3(grid), dim3(WNT), kLds4 + kLdsExtra, stream, a); break;
    default: hipLaunchKernelGGL((k_gemm_w4<1, 1>), dim3(grid), dim3(WNT), kLds4 + kLdsExtra, stream, a); break;
  }
}

int gemm_w4_tiles(int M, int N) { return ((M + WM - 1) / WM) * ((N + WNB - 1) / WNB); }

void launch_gemm_nt_w4_fused(const GemmArgs& g, const FusedArgs& f, hipStream_t stream) {
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }();
  // one workgroup per tile (the persistent form spills registers with the fused epilogue)
  static bool attr = [] {
    w4_attr(reinterpret_cast<const void*>(k_gemm_w4<0, 0, 1>));
    return true;
  }();
  (void)attr;
  (void)cus;
  const int ntiles = gemm_w4_tiles(g.M, g.N);
  W4Args a{g, g_w4_group_m, f, nullptr};
  hipLaunchKernelGGL((k_gemm_w4<0, 0, 1>), dim3(ntiles), dim3(WNT), kLds4 + kLdsExtra, stream, a);
}

void launch_fused_wait(const FusedArgs& f, int tiles, hipStream_t stream) {
  hipLaunchKernelGGL(k_fused_wait, dim3(1), dim3(256), 0, stream, f, tiles);
}

}  // namespace gemm
}  // namespace dev
}  // namespace ccmpi
