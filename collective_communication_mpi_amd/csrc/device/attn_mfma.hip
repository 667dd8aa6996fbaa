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
#include <hip/hip_runtime.h>

#include <algorithm>

#include "attn_common.hpp"
#include "common.hpp"

namespace ccmpi {
namespace dev {
namespace attn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int WPB = 4;  // waves per workgroup

__device__ __forceinline__ s4 pack4(float a, float b, float c, float d) {
  const uint2 u{f32_to_bf16_bits(a) | (f32_to_bf16_bits(b) << 16), f32_to_bf16_bits(c) | (f32_to_bf16_bits(d) << 16)};
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

template <int D>
__global__ void __launch_bounds__(256) k_attn16_fwd(AttnArgs a) {
  constexpr int LD = D + 8, NK = D / 32, NT = D / 16;
  __shared__ __attribute__((aligned(16))) uint16_t vt[WPB][16 * LD];
  __shared__ __attribute__((aligned(16))) uint16_t ot[WPB][16 * LD];
  __shared__ float zpart[2][WPB][16];  // fused fc_o: per-wave (= per-head) partial logits, double-buffered
  // per-token fused fc_o: per-wave (= per-head) z tiles [16 tokens][16 classes], double-buffered
  __shared__ float ztp[2][WPB][16 * 16];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int S = a.S, HD = a.Hl * D, npairs = a.B * a.Hl;
  uint16_t* V = vt[wave];
  uint16_t* O = ot[wave];
  // workgroup-uniform trip count (the fused fc_o reduces across the waves of an iteration);
  // with Hl | WPB the Hl heads of a sequence are consecutive waves of one workgroup
  // fused fc_o: with Hl | WPB this wave always serves head h = wave % Hl, so its W_o
  // entries (classes 4g..4g+3, features 16nt + c) are loaded once, packed as bf16 pairs
  uint32_t wpk[NT][2];
  if (a.zp) {
    const int hw = wave % a.Hl;
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
  bf16x8 wb[NK];
  if (a.ztok || a.zrows) {
    const int hw = wave % a.Hl;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
      wb[kk] = ld_row16(a.wo + (size_t)c * a.ld_wo + hw * D + 32 * kk + 8 * g, c < a.n_out);
  }
  const int stride = gridDim.x * WPB;
  int it = 0;
  for (int base = blockIdx.x * WPB; base < npairs; base += stride, it ^= 1) {
   const int pr = base + wave;
   if (pr < npairs) {
    const int b = pr / a.Hl, h = pr % a.Hl;
    bf16x8 qr[NK], kr[NK];
    {
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
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float e[4], s = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      e[r] = __expf(x[r] - m);
      s += e[r];
    }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    const float inv = 1.f / s;
    if (g == 0 && c < S) a.lse[(size_t)pr * S + c] = m + __logf(s);
    const s4 pa = pack4(e[0] * inv, e[1] * inv, e[2] * inv, e[3] * inv);  // A[i = c][j = 4g + jj]
    __builtin_amdgcn_wave_barrier();
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
        cs += __shfl_xor(cs, 16);
        cs += __shfl_xor(cs, 32);
        const uint32_t pb = f32_to_bf16_bits(cs / (float)S);
        if (g == 0) a.pool[(size_t)b * a.ld_pool + h * D + 16 * nt + c] = (uint16_t)pb;
        if (a.zp) {
          const float pv = __uint_as_float(pb << 16);  // the bf16 value a separate fc_o GEMM would read
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            zacc[2 * q] += pv * bf16_lo(wpk[nt][q]);
            zacc[2 * q + 1] += pv * bf16_hi(wpk[nt][q]);
          }
        }
      }
      if (a.zp) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float acc = zacc[j];
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) acc += __shfl_xor(acc, off);
          if (c == 0) zpart[it][wave][4 * g + j] = acc;
        }
      }
    }
    if (a.ztok || a.zrows) {
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
   }
   if (a.ztok || a.zrows) {
    // the Hl heads of each sequence of this iteration (consecutive waves, Hl | WPB), summed in
    // head order, + the bias.  Wave s writes sequence s (waves s >= WPB / Hl idle): lane l =
    // (token l >> 2, classes 4 (l & 3) .. +3), one 16-B store per lane, a sequence's S x 16
    // fp32 rows as whole lines
    __syncthreads();  // (the next iteration writes the other buffer)
    const int i = lane >> 2, q = (lane & 3) * 4, w = wave * a.Hl;
    const int prw = base + w;
    if (w < WPB && prw < npairs) {
      const int b = prw / a.Hl;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (a.bo && q + r < a.n_out) ? a.bo[q + r] : 0.f;
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
        } else {
          *reinterpret_cast<u32x4*>(a.ztok + (row0 + i) * a.ld_zt + q) = pk;
        }
      }
    }
   }
   if (a.zp) {  // sum the Hl heads of each sequence in rank order (deterministic) and add the bias
    __syncthreads();  // (the next iteration writes the other buffer: one barrier per iteration)
    const int t = threadIdx.x, w = t >> 4, cls = t & 15, prw = base + w;
    if (t < WPB * 16 && prw < npairs && prw % a.Hl == 0 && cls < a.n_out) {
      float acc = 0.f;
      for (int k = 0; k < a.Hl; ++k) acc += zpart[it][w + k][cls];
      if (a.bo) acc += a.bo[cls];
      a.zp[(size_t)(prw / a.Hl) * a.ld_zp + cls] = acc;
    }
   }
  }
}


// Fused QKV projection + attention + per-token fc_o (the harness forward, fc_o_mode "token"):
// one wave per sequence (S <= 16 tokens), looping over the Hl local heads.  Per head the
// workgroup stages that head's rows of the folded QKV weight (3 D rows x kq <= 96 columns,
// bf16) in LDS; each wave forms its sequence's q | k | v = X W_h^T + b on the MFMA (X = the
// sequence's patch rows, the A operand read straight from global memory, zero past kq),
// rounds them to bf16 into its LDS tile (the values the unfused QKV GEMM would store), runs
// the attention of k_attn16_fwd on them, and adds this head's share of z = O W_o^T to one
// MFMA accumulator chained over the heads (heads summed in head order).  The qkv tensor's
// write + read (2 x B*S x 3 Hl D x 2 B) and the QKV GEMM launch disappear; qkv is stored only
// when a backward needs it (qkv_out).  z rows go to ztok or, pushed, to the TP owners' inbox
// slots (zrows), as in k_attn16_fwd.
template <int D>
__global__ void __launch_bounds__(256) k_qkv_attn16_fwd(AttnArgs a) {
  constexpr int NK = D / 32, NT = D / 16;
  constexpr int KQ = 96;           // projection depth: kq <= 96 columns, 3 MFMA k-steps
  constexpr int LDW = KQ + 8;      // staged W row (bf16)
  constexpr int LDT = 3 * D + 8;   // per-wave q | k | v tile row (bf16)
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  uint16_t* W = sm;  // [3 D][LDW]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  uint16_t* T = sm + 3 * D * LDW + wave * 16 * LDT;  // [16][LDT]
  const int S = a.S, HD = a.Hl * D;
  const int stride = gridDim.x * WPB;
  for (int base = blockIdx.x * WPB; base < a.B; base += stride) {  // workgroup-uniform trip count
    const int b = base + wave;
    const bool live = b < a.B;
    bf16x8 xr[3];  // patch rows: lane (c, g) holds token c, columns 32 kk + 8 g .. +7
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      const int col = 32 * kk + 8 * g;
      xr[kk] = ld_row16(a.xq + (size_t)(live ? b * S + c : 0) * a.ld_xq + col, live && c < S && col < a.kq);
    }
    f4 zt = {0.f, 0.f, 0.f, 0.f};
    for (int h = 0; h < a.Hl; ++h) {
      __syncthreads();  // every wave is done with the previous head's W tile
      for (int q = threadIdx.x; q < 3 * D * (KQ / 8); q += blockDim.x) {
        const int row = q / (KQ / 8), col = (q % (KQ / 8)) * 8, sel = row / D, f = row % D;
        uint4 v = {0u, 0u, 0u, 0u};
        if (col < a.kq) v = *reinterpret_cast<const uint4*>(a.wq + (size_t)(sel * HD + h * D + f) * a.ld_wq + col);
        *reinterpret_cast<uint4*>(W + row * LDW + col) = v;
      }
      __syncthreads();
      if (!live) continue;
      // q | k | v of head h: acc[r] = out[token 4 g + r][feature 16 nt + c] (+ bias, bf16)
#pragma unroll
      for (int sel = 0; sel < 3; ++sel)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < 3; ++kk)
            acc = mma32(xr[kk], *reinterpret_cast<const bf16x8*>(W + (sel * D + 16 * nt + c) * LDW + 32 * kk + 8 * g),
                        acc);
          const float bias = a.bq[sel * HD + h * D + 16 * nt + c];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            T[(4 * g + r) * LDT + sel * D + 16 * nt + c] = (uint16_t)f32_to_bf16_bits(acc[r] + bias);
        }
      __builtin_amdgcn_wave_barrier();
      if (a.qkv_out) {  // the projection for a backward: rows < S, 16-B vectors
        for (int p = lane; p < 16 * 3 * (D / 8); p += 64) {
          const int row = p / (3 * (D / 8)), rem = p % (3 * (D / 8)), sel = rem / (D / 8), ch = rem % (D / 8);
          if (row < S)
            *reinterpret_cast<uint4*>(a.qkv_out + (size_t)(b * S + row) * a.ld_qkv + sel * HD + h * D + ch * 8) =
                *reinterpret_cast<const uint4*>(T + row * LDT + sel * D + ch * 8);
        }
      }
      bf16x8 qr[NK], kr[NK];
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        qr[kk] = *reinterpret_cast<const bf16x8*>(T + c * LDT + 32 * kk + 8 * g);
        kr[kk] = *reinterpret_cast<const bf16x8*>(T + c * LDT + D + 32 * kk + 8 * g);
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
      m = fmaxf(m, __shfl_xor(m, 16));
      m = fmaxf(m, __shfl_xor(m, 32));
      float e[4], ssum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        e[r] = __expf(x[r] - m);
        ssum += e[r];
      }
      ssum += __shfl_xor(ssum, 16);
      ssum += __shfl_xor(ssum, 32);
      const float inv = 1.f / ssum;
      const int pr = b * a.Hl + h;
      if (g == 0 && c < S) a.lse[(size_t)pr * S + c] = m + __logf(ssum);
      const s4 pa = pack4(e[0] * inv, e[1] * inv, e[2] * inv, e[3] * inv);
      f4 o[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) o[nt] = mma16(pa, tile_b<LDT>(T + 2 * D, g, 16 * nt + c), f4{0.f, 0.f, 0.f, 0.f});
      if (a.pool) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          float cs = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) cs += (4 * g + r < S) ? o[nt][r] : 0.f;
          cs += __shfl_xor(cs, 16);
          cs += __shfl_xor(cs, 32);
          if (g == 0) a.pool[(size_t)b * a.ld_pool + h * D + 16 * nt + c] = (uint16_t)f32_to_bf16_bits(cs / (float)S);
        }
      }
      // z += bf16(O_h) W_o,h^T: O staged over the tile's (dead) q columns, the A operand
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(4 * g + r) * LDT + 16 * nt + c] = (uint16_t)f32_to_bf16_bits(o[nt][r]);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const bf16x8 wb = ld_row16(a.wo + (size_t)c * a.ld_wo + h * D + 32 * kk + 8 * g, c < a.n_out);
        zt = mma32(*reinterpret_cast<const bf16x8*>(T + c * LDT + 32 * kk + 8 * g), wb, zt);  // z[4g + r][c]
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (live) {
      // + the bias, then whole 64-B rows: stage z as fp32 [16][16] in the tile
      float* Z = reinterpret_cast<float*>(T);
      const float bo = (a.bo && c < a.n_out) ? a.bo[c] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) Z[(4 * g + r) * 16 + c] = zt[r] + bo;
      __builtin_amdgcn_wave_barrier();
      const int i = lane >> 2, q = (lane & 3) * 4;
      const u32x4 pk = *reinterpret_cast<const u32x4*>(Z + i * 16 + q);
      const size_t row0 = (size_t)b * S;
      if (i < S) {
        if (a.zrows) {
          const int j = __builtin_amdgcn_readfirstlane((int)(row0 / a.zrows));
          char* seq = reinterpret_cast<char*>(a.zpush[j] + (row0 - (size_t)j * a.zrows) * a.ld_zt);
          const Rsrc rs = make_rsrc(uniform_ptr(seq), (uint32_t)(S * a.ld_zt * 4));
          __builtin_amdgcn_raw_buffer_store_b128(pk, rs.r, (uint32_t)((i * a.ld_zt + q) * 4), 0, kStorePolicy);
        } else {
          *reinterpret_cast<u32x4*>(a.ztok + (row0 + i) * a.ld_zt + q) = pk;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

template <int D>
constexpr size_t qkv_fwd_lds_bytes() {
  return (size_t)(3 * D * (96 + 8) + WPB * 16 * (3 * D + 8)) * sizeof(uint16_t);
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
    dl += __shfl_xor(dl, 16);        // ... and across the four lane groups
    dl += __shfl_xor(dl, 32);
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
      q += __shfl_xor(q, 16); q += __shfl_xor(q, 32);
      k += __shfl_xor(k, 16); k += __shfl_xor(k, 32);
      v += __shfl_xor(v, 16); v += __shfl_xor(v, 32);
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

int grid_for(int npairs, int cap) { return std::max(1, std::min((npairs + WPB - 1) / WPB, cap)); }

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

void launch_qkv_fwd_mfma(const AttnArgs& a, hipStream_t stream) {
  const int grid = grid_for(a.B, 4096);
  auto go = [&](const void* k, size_t lds) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  };
  if (a.D == 32) {
    static bool attr = (go(reinterpret_cast<const void*>(k_qkv_attn16_fwd<32>), qkv_fwd_lds_bytes<32>()), true);
    (void)attr;
    hipLaunchKernelGGL(k_qkv_attn16_fwd<32>, dim3(grid), dim3(256), qkv_fwd_lds_bytes<32>(), stream, a);
  } else if (a.D == 64) {
    static bool attr = (go(reinterpret_cast<const void*>(k_qkv_attn16_fwd<64>), qkv_fwd_lds_bytes<64>()), true);
    (void)attr;
    hipLaunchKernelGGL(k_qkv_attn16_fwd<64>, dim3(grid), dim3(256), qkv_fwd_lds_bytes<64>(), stream, a);
  } else {
    static bool attr = (go(reinterpret_cast<const void*>(k_qkv_attn16_fwd<128>), qkv_fwd_lds_bytes<128>()), true);
    (void)attr;
    hipLaunchKernelGGL(k_qkv_attn16_fwd<128>, dim3(grid), dim3(256), qkv_fwd_lds_bytes<128>(), stream, a);
  }
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
