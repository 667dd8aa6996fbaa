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
  return f32_to_bf16_bits(a) | (f32_to_bf16_bits(b) << 16);
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
            for (int q = 0; q < 4; ++q) w[q] = f32_to_bf16_bits(v[2 * q]) | (f32_to_bf16_bits(v[2 * q + 1]) << 16);
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
// Ring variant (profiles/r3_gemm_ring): the same 256x256 tile and 128x128 wave tiles,
// but LDS is a ring of four 32-KiB slots, each one 32-deep K-step (A 256 x 64 B |
// B 256 x 64 B).  A phase is one K-step: 64 MFMAs on the previous step's fragments,
// 16 fragment reads of this step, and the 8 DMA pieces of the step THREE ahead (into
// the slot read two phases ago), then a counted `s_waitcnt vmcnt(16)` (the next step
// landed, the two after it still in flight) + lgkmcnt(0) + a raw s_barrier.  The
// two-stage kernel above waits vmcnt(0) at every barrier, so the DMA of a K-tile has
// one phase to land; PMC counters of it against hipBLASLt on the same shape showed 6x
// the wave wait cycles at equal instruction counts (profiles/r3_gemm_pmc).
//
// 64-B rows: 16-B chunk c of row r sits at physical chunk c ^ f((r >> 2) & 3),
// f = {0, 2, 3, 1}: conflict-free for the 16x16x32 fragment reads (ds_read_b128 lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... each cover the 16 slots of a
// 256-B bank row).  The DMA keeps LDS lane-linear and permutes the source chunk.
constexpr int kRing = 32768;   // one ring slot
constexpr int kRingHalf = 16384;
__device__ __forceinline__ int ring_swz(int q) { return (0x78 >> (2 * q)) & 3; }

__device__ __forceinline__ void wait_barrier_ring(int later) {
  // `later` DMA steps (8 pieces each) may stay in flight past this barrier
  if (later >= 2) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (later == 1) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int PRIO>
__global__ void __launch_bounds__(WNT, 1) k_gemm_w4r(W4Args wa) {
  const GemmArgs& g = wa.g;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tiles_n = (g.N + WNB - 1) / WNB, tiles_m = (g.M + WM - 1) / WM;
  const int lt = xcd_remap(blockIdx.x, gridDim.x);
  if (lt >= tiles_n * tiles_m) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nst = g.K / 32;
  int tm, tn;
  tile_coords(lt, tiles_m, tiles_n, wa.group_m, tm, tn);
  const int bm = tm * WM, bn = tn * WNB;
  const __amdgpu_buffer_rsrc_t ra = op_rsrc(g.A + (size_t)bm * g.lda, (long)g.M - bm, g.lda);
  const __amdgpu_buffer_rsrc_t rb = op_rsrc(g.B + (size_t)bn * g.ldb, (long)g.N - bn, g.ldb);

  // DMA piece i of a step: 16 rows x 64 B; wave w covers rows (4 i + w) * 16 ..
  // lane l: row + (l >> 2), physical chunk l & 3 <- logical chunk (l & 3) ^ f((l >> 4) & 3)
  const int drow = wave * 16 + (lane >> 2);
  const int dchunk = ((lane & 3) ^ ring_swz((lane >> 4) & 3)) << 4;
  const int va = drow * g.lda * 2 + dchunk, vb = drow * g.ldb * 2 + dchunk;
  auto dma = [&](int s, int i) {
    int sa_ = 64 * g.lda * 2, sb_ = 64 * g.ldb * 2;
    asm volatile("" : "+s"(sa_), "+s"(sb_));
    unsigned char* base = smem + (s & 3) * kRing + wave * 1024;
    const int k0 = s * 64;
    if (i < 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_vptr)(base + i * 4096), 16, va, k0 + i * sa_, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_vptr)(base + kRingHalf + (i - 4) * 4096), 16, vb,
                                               k0 + (i - 4) * sb_, 0, 0);
  };
  // fragment (16x16x32): lane l reads row (l & 15) of a 16-row block, logical chunk l >> 4;
  // the physical chunk depends on the lane only (block rows are multiples of 16)
  const int rdo = (lane & 15) * 64 + (((lane >> 4) ^ ring_swz((lane >> 2) & 3)) << 4);
  // group grp (0..7) of a phase reads B blocks 2 grp, 2 grp + 1 (grp < 4), then A blocks
  auto rd2 = [&](int s, int grp, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const unsigned char* base = smem + (s & 3) * kRing + (grp < 4 ? kRingHalf : 0) + rdo;
    const int r0 = (grp < 4 ? wc : wr) * 128 + (grp & 3) * 32;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(base + (r0 + u * 16) * 64);
      if (grp < 4) fb[(grp & 3) * 2 + u] = v;
      else fa[(grp & 3) * 2 + u] = v;
    }
  };

  floatx4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];

  // one phase: MFMAs on (pa, pb) = step q-1, reads of step q into (ca, cb), DMA of step
  // q+3 (DMA), then the barrier with LATER steps still in flight (branch-free body)
  auto phase = [&](auto dma_c, auto later_c, int q, const bf16x8 (&pa)[8], const bf16x8 (&pb)[8],
                   bf16x8 (&ca)[8], bf16x8 (&cb)[8]) {
    constexpr bool DMA = decltype(dma_c)::value;
    constexpr int LATER = decltype(later_c)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[i], pb[j], acc[i][j], 0, 0, 0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      rd2(q, i, ca, cb);
      if constexpr (DMA) dma(q + 3, i);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_barrier_ring(LATER);
  };
  using T = std::true_type;
  using F = std::false_type;
  using L2 = std::integral_constant<int, 2>;
  using L1 = std::integral_constant<int, 1>;
  using L0 = std::integral_constant<int, 0>;

  // prologue: steps 0..2 in flight (nst is even: 2 or >= 4), step 0 landed; then
  // "phase 0": step 0's fragments read, step 3 into the last free slot, step 1 landed
  const int pro = min(nst, 3);
  for (int s = 0; s < pro; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) dma(s, i);
  wait_barrier_ring(pro - 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    rd2(0, i, a0, b0);
    if (nst >= 4) dma(3, i);
  }
  wait_barrier_ring(nst >= 4 ? 2 : 0);
  // steady state: phases 1 .. nst-4 in pairs, each prefetching the step three ahead
  for (int q = 1; q + 3 < nst; q += 2) {
    phase(T{}, L2{}, q, a0, b0, a1, b1);
    phase(T{}, L2{}, q + 1, a1, b1, a0, b0);
  }
  if (nst >= 4) {  // drain: phases nst-3, nst-2, nst-1
    phase(F{}, L1{}, nst - 3, a0, b0, a1, b1);
    phase(F{}, L0{}, nst - 2, a1, b1, a0, b0);
  }
  phase(F{}, L0{}, nst - 1, a0, b0, a1, b1);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);

  // ---- epilogue (the ring is idle: the last barrier saw every read and DMA retire)
  float* tile = reinterpret_cast<float*>(smem + wave * kEpiWave);
  const int cl = (lane & 15) * 8;
  const int col = bn + wc * 128 + cl;
  float bias[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bias[q] = load_bias(g, col + q, 0);
  const int es = g.out_bf16 ? 2 : 4;
  const bool vec_ok = (((uint64_t)g.C | ((uint64_t)g.ldc * es)) % 16) == 0 && g.N % 8 == 0;
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
          for (int q = 0; q < 4; ++q) w[q] = f32_to_bf16_bits(v[2 * q]) | (f32_to_bf16_bits(v[2 * q + 1]) << 16);
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
}

}  // namespace

int g_w4_sched = 1;   // bit 0: persistent grid, bit 1: MFMA-first order inside groups, bit 2: front-loaded DMA,
                      // bit 3: ring kernel (k_gemm_w4r; bit 4 with s_setprio around the MFMA groups)
int g_w4_group_m = 8;

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

void launch_gemm_nt_w4(const GemmArgs& g, hipStream_t stream) {
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }();
  const int ntiles = ((g.M + WM - 1) / WM) * ((g.N + WNB - 1) / WNB);
  W4Args a{g, g_w4_group_m, {}};
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
    static bool rattr = [] {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_w4r<0>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kRing);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_w4r<1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kRing);
      return true;
    }();
    (void)rattr;
    if (g_w4_sched & 16) hipLaunchKernelGGL(k_gemm_w4r<1>, dim3(ntiles), dim3(WNT), 4 * kRing, stream, a);
    else hipLaunchKernelGGL(k_gemm_w4r<0>, dim3(ntiles), dim3(WNT), 4 * kRing, stream, a);
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
  W4Args a{g, g_w4_group_m, f};
  hipLaunchKernelGGL((k_gemm_w4<0, 0, 1>), dim3(ntiles), dim3(WNT), kLds4 + kLdsExtra, stream, a);
}

void launch_fused_wait(const FusedArgs& f, int tiles, hipStream_t stream) {
  hipLaunchKernelGGL(k_fused_wait, dim3(1), dim3(256), 0, stream, f, tiles);
}

}  // namespace gemm
}  // namespace dev
}  // namespace ccmpi
