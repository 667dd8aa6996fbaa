// Shared pieces of the MFMA GEMM kernels (gemm.hip, gemm256.hip): argument
// block, epilogue math and the LDS-staged row store.
#pragma once
#include <cstdint>

#include "common.hpp"

namespace ccmpi {
namespace dev {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const void* bias;
  int M, N, K;
  int lda, ldb, ldc;
  float alpha;
  int accumulate;  // C += result
  int bias_kind;   // 0 none, 1 fp32, 2 bf16
  int act;         // 0 none, 1 relu, 2 gelu(tanh)
  int out_bf16;    // 0 fp32 out, 1 bf16 out
  int splitk;      // >1: K split over workgroups, fp32 atomic-add epilogue into C
};

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

__device__ __forceinline__ float load_bias(const GemmArgs& g, int col, int split) {
  if (split != 0 || col >= g.N) return 0.f;
  if (g.bias_kind == 1) return reinterpret_cast<const float*>(g.bias)[col];
  if (g.bias_kind == 2) return bf2f(reinterpret_cast<const uint16_t*>(g.bias)[col]);
  return 0.f;
}

__device__ __forceinline__ float epi(const GemmArgs& g, float acc, float b) {
  float v = g.alpha * acc + b;
  if (g.act == 1) v = fmaxf(v, 0.f);
  else if (g.act == 2) v = gelu_tanh(v);
  return v;
}

// Write a ROWS x COLS fp32 tile staged in LDS (row stride TS floats, values
// already alpha/bias/act-applied) to C at (row0, col0) with NT threads: whole
// rows as 16-B vectors when C allows it, lane-consecutive fp32 atomics for
// split-K, per-element stores otherwise.
template <int ROWS, int COLS, int NT>
__device__ __forceinline__ void store_rows(const GemmArgs& g, const float* tile, int TS, int row0, int col0, int t) {
  const int es = g.out_bf16 ? 2 : 4;
  const bool vec_ok = (((uint64_t)g.C | ((uint64_t)g.ldc * es)) % 16) == 0;
  if (g.splitk > 1) {
    for (int idx = t; idx < ROWS * COLS; idx += NT) {
      const int rl = idx / COLS, cl = idx % COLS;
      const int row = row0 + rl, col = col0 + cl;
      if (row < g.M && col < g.N) atomicAdd(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col, tile[rl * TS + cl]);
    }
  } else if (vec_ok) {
    const int per_vec = 16 / es;
    const int vecs_row = COLS / per_vec;
    for (int idx = t; idx < ROWS * vecs_row; idx += NT) {
      const int rl = idx / vecs_row, cl = (idx % vecs_row) * per_vec;
      const int row = row0 + rl, col = col0 + cl;
      if (row >= g.M || col >= g.N) continue;
      const float* src = tile + rl * TS + cl;
      if (col + per_vec <= g.N) {
        if (g.out_bf16) {
          uint16_t* C = reinterpret_cast<uint16_t*>(g.C) + (size_t)row * g.ldc + col;
          uint32_t w[4];
          if (g.accumulate) {
            const uint4 old = *reinterpret_cast<const uint4*>(C);
            const uint32_t ow[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
              w[q] = pk_bf16(src[2 * q] + bf16_lo(ow[q]), src[2 * q + 1] + bf16_hi(ow[q]));
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) w[q] = pk_bf16(src[2 * q], src[2 * q + 1]);
          }
          *reinterpret_cast<uint4*>(C) = uint4{w[0], w[1], w[2], w[3]};
        } else {
          float* C = reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col;
          float4 v = make_float4(src[0], src[1], src[2], src[3]);
          if (g.accumulate) {
            const float4 old = *reinterpret_cast<const float4*>(C);
            v.x += old.x; v.y += old.y; v.z += old.z; v.w += old.w;
          }
          *reinterpret_cast<float4*>(C) = v;
        }
      } else {
        for (int q = 0; q < per_vec && col + q < g.N; ++q) {
          const size_t o = (size_t)row * g.ldc + col + q;
          if (g.out_bf16) {
            uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
            C[o] = (uint16_t)f32_to_bf16_bits(src[q] + (g.accumulate ? bf2f(C[o]) : 0.f));
          } else {
            float* C = reinterpret_cast<float*>(g.C);
            C[o] = src[q] + (g.accumulate ? C[o] : 0.f);
          }
        }
      }
    }
  } else {
    for (int idx = t; idx < ROWS * COLS; idx += NT) {
      const int rl = idx / COLS, cl = idx % COLS;
      const int row = row0 + rl, col = col0 + cl;
      if (row >= g.M || col >= g.N) continue;
      const size_t o = (size_t)row * g.ldc + col;
      const float v = tile[rl * TS + cl];
      if (g.out_bf16) {
        uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
        C[o] = (uint16_t)f32_to_bf16_bits(v + (g.accumulate ? bf2f(C[o]) : 0.f));
      } else {
        float* C = reinterpret_cast<float*>(g.C);
        C[o] = v + (g.accumulate ? C[o] : 0.f);
      }
    }
  }
}

// Branch-free form of store_rows for the common case (no split-K, no
// accumulate, 16-B aligned C, N % 8 == 0): whole 16-B row vectors only.
template <int ROWS, int COLS, int NT, bool OUT_BF16>
__device__ __forceinline__ void store_rows_fast(const GemmArgs& g, const float* tile, int TS, int row0, int col0, int t) {
  constexpr int per_vec = OUT_BF16 ? 8 : 4;
  constexpr int vecs_row = COLS / per_vec;
  for (int idx = t; idx < ROWS * vecs_row; idx += NT) {
    const int rl = idx / vecs_row, cl = (idx % vecs_row) * per_vec;
    const int row = row0 + rl, col = col0 + cl;
    if (row >= g.M || col >= g.N) continue;
    const float* src = tile + rl * TS + cl;
    if constexpr (OUT_BF16) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = pk_bf16(src[2 * q], src[2 * q + 1]);
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(g.C) + (size_t)row * g.ldc + col) = uint4{w[0], w[1], w[2], w[3]};
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col) =
          make_float4(src[0], src[1], src[2], src[3]);
    }
  }
}

// Fast-epilogue id shared by the kernels: 1 + out_bf16 + 2 * bias_kind when the
// epilogue needs no split-K, accumulate, activation or unaligned stores; 0 otherwise.
inline int fast_epilogue_id(const GemmArgs& g) {
  const int es = g.out_bf16 ? 2 : 4;
  const bool ok = g.splitk == 1 && !g.accumulate && g.act == 0 && g.N % 8 == 0 &&
                  (((uint64_t)g.C | ((uint64_t)g.ldc * es)) % 16) == 0;
  return ok ? 1 + (g.out_bf16 ? 1 : 0) + 2 * g.bias_kind : 0;
}

// XCD-aware bijective workgroup remap: blocks b, b+8, b+16, ... (dispatched
// round-robin to the same XCD) get consecutive logical ids.
__device__ __forceinline__ int xcd_remap(int wg, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = wg % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / 8;
}

// ---- row-parallel GEMM with the TP all-reduce fused into its epilogue (gemm_w4.hip) ----
// Every rank computes the same output tiles from its K-shard.  Per tile, each rank
// draws a ticket from the tile owner's counter (owner = tile % p); the first p - 1
// arrivals store their bf16 partial into the owner's inbox slot and flag it, the
// last arrival sums all partials in rank order (its own from registers, rounded to
// bf16 like the others, so the sum does not depend on who arrives last), adds the
// bias and writes the final tile into every rank's output, then flags it done on
// every rank.  Nobody waits for a workgroup that has not started (the last arrival
// waits only for ticket holders), so it cannot deadlock when ranks share a GPU.
constexpr int kFusedMaxTiles = 4096;
constexpr uint64_t kFusedTileBytes = 256ull * 256 * 2;  // one bf16 256 x 256 partial
struct FusedState {                        // per rank, uncached, peer-mapped
  uint64_t out_code[2];                    // [0] this call's output (addr_code), [1] its call sequence
  uint64_t pad[6];
  uint32_t cnt[kFusedMaxTiles];            // owner: tickets drawn for tile t (reset by its reducer)
  uint64_t ready[kFusedMaxTiles][kMaxRanks];  // owner: slot (t, j) holds call `value`'s partial
  uint64_t done[kFusedMaxTiles];           // every rank: tile t of call `value` is final here
};
struct FusedTable {                        // device-resident, per group (set up once)
  FusedState* state[kMaxRanks];            // state[j]: rank j's (mapped)
  uint64_t inbox_code[kMaxRanks];          // rank j's inbox (>= ceil(T / p) * p tile slots)
};
struct FusedArgs {
  const PeerTable* pt;
  const FusedTable* tab;
  uint64_t out_code;                       // this rank's output
  uint64_t seq;                            // call sequence number (identical on every rank)
  uint64_t timeout_ticks;
};
void launch_gemm_nt_w4_fused(const GemmArgs& g, const FusedArgs& f, hipStream_t stream);
// one workgroup: wait until every tile of call `seq` is done on this rank (bounded)
void launch_fused_wait(const FusedArgs& f, int tiles, hipStream_t stream);
int gemm_w4_tiles(int M, int N);

// 256 x bn (bn = 256 or 128) 8-wave ping-pong kernel (gemm256.hip); requires K % 128 == 0.
void launch_gemm_nt_256(const GemmArgs& g, int bn, hipStream_t stream);
int gemm256_tiles(int M, int N, int bn);
extern int g_pp_exp;
// TN (weight-gradient) form of the 256x256 ping-pong kernel; K (reduction rows) % 128 == 0,
// N1, N2 % 8 == 0.  splitk > 1: g.C is a workspace of splitk fp32 [N1][N2] slices.
void launch_gemm_tn_256(const GemmArgs& g, hipStream_t stream);
// 256 x 256 four-wave kernel (gemm_w4.hip): 128 x 128 per wave, K % 64 == 0, no split-K
bool gemm_w4_ok(const GemmArgs& g);
extern int g_pair_nobar;  // diagnostic: pair ring without its odd-phase barrier (wrong results)
extern int g_pair_ta;     // K-major A alone on the pair-slot ring (CCMPI_PAIR_TA; gemm_set_pair_ta)
extern int g_ring_sched;  // auto-dispatched LDS-ring kernel variant (gemm_w4.hip launch_gemm_ring)
extern long long g_ring_launches;  // launch_gemm_ring calls (tests: the ring path really ran)
extern int g_w4_sched;    // four-wave kernel variant: bit 0 persistent grid, bit 1 MFMA-first group order
extern unsigned long long* g_w4_dbg;  // four-wave ring STAMP diagnostic output (benchmarks)
extern int g_w4_group_m;  // four-wave kernel: tile rows per group-M block
void launch_gemm_nt_w4(const GemmArgs& g, hipStream_t stream);
bool gemm_w4r_fast(const GemmArgs& g);  // the LDS-ring kernel's fast epilogue applies
void launch_gemm_nt_w4r(const GemmArgs& g, hipStream_t stream);  // LDS-ring kernel (sched bits from g_w4_sched)
// LDS-ring kernel with operand layouts: ta / tb = 1 reads A / B K-major ([K][M] / [K][N])
bool gemm_ring_ok(const GemmArgs& g, int ta, int tb);
// push / push_rows: EPI 1 stores output row block j (push_rows rows) at push[j] instead of C
void launch_gemm_ring(const GemmArgs& g, int ta, int tb, hipStream_t stream, uint16_t* glu = nullptr, int ldglu = 0,
                      uint16_t* const* push = nullptr, int push_rows = 0);
extern long long g_ring_min_macs;  // gemm_nt auto: the LDS-ring kernel from this many MACs up (0 = never)  // ablation variant of the ping-pong kernel (benchmarks only; 0 = production)

}  // namespace gemm
}  // namespace dev
}  // namespace ccmpi
