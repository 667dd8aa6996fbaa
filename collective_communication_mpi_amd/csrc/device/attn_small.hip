// Fused attention for short sequences (the MNIST harness: S = 16 patches,
// head_dim 64), forward and backward, one workgroup per (batch, local head).
//
// Inputs come straight from the fused QKV GEMM output [B*S][3*Hl*D] (q | k | v
// column blocks, head h at columns h*D..h*D+D-1 of each block) so no split /
// transpose / contiguous copies are needed; the output [B*S][Hl*D] is exactly
// the row-parallel fc_o's input layout.  The whole S x S score tile lives in
// LDS, so the softmax is exact (no online rescaling) and the log-sum-exp is
// stored for the backward recompute.  At S <= 64 the S x S x D products are a
// few thousand FMAs per head: the kernel is load/latency bound, so it uses
// fp32 VALU dot products from LDS rather than MFMA tiles (which need >= 16x16x32).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <tuple>
#include <vector>

#include "attn_common.hpp"
#include "common.hpp"
#include "ops.hpp"

namespace ccmpi {
namespace dev {

namespace {
using attn::AttnArgs;

__device__ __forceinline__ float ld_bf16(const uint16_t* p) { return __uint_as_float((uint32_t)(*p) << 16); }
__device__ __forceinline__ void st_bf16(uint16_t* p, float v) { *p = (uint16_t)f32_to_bf16_bits(v); }

__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}



// stage an S x D head tile (bf16, row stride ld) into fp32 LDS [S][D+1]; 16-B
// vector loads (8 bf16 per lane) whenever rows are 16-B aligned (guide G13)
__device__ __forceinline__ void stage(float* dst, const uint16_t* src, int S, int D, int ld) {
  if ((D % 8) == 0 && (ld % 8) == 0 && ((uint64_t)src % 16) == 0) {
    const int vr = D / 8;
    for (int idx = threadIdx.x; idx < S * vr; idx += blockDim.x) {
      const int i = idx / vr, c = (idx % vr) * 8;
      const uint4 w = *reinterpret_cast<const uint4*>(src + (size_t)i * ld + c);
      float* o = dst + i * (D + 1) + c;
      o[0] = bf16_lo(w.x); o[1] = bf16_hi(w.x); o[2] = bf16_lo(w.y); o[3] = bf16_hi(w.y);
      o[4] = bf16_lo(w.z); o[5] = bf16_hi(w.z); o[6] = bf16_lo(w.w); o[7] = bf16_hi(w.w);
    }
    return;
  }
  for (int idx = threadIdx.x; idx < S * D; idx += blockDim.x) {
    const int i = idx / D, d = idx % D;
    dst[i * (D + 1) + d] = ld_bf16(src + (size_t)i * ld + d);
  }
}

__global__ void __launch_bounds__(256) k_attn_fwd(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int S = a.S, D = a.D, Dp = D + 1, Sp = S + 1;
  const int b = blockIdx.x / a.Hl, h = blockIdx.x % a.Hl;
  float* q = sm;
  float* k = q + S * Dp;
  float* v = k + S * Dp;
  float* P = v + S * Dp;
  const uint16_t* base = a.qkv + (size_t)b * S * a.ld_qkv + h * D;
  const int HD = a.Hl * D;
  stage(q, base, S, D, a.ld_qkv);
  stage(k, base + HD, S, D, a.ld_qkv);
  stage(v, base + 2 * HD, S, D, a.ld_qkv);
  __syncthreads();
  for (int idx = threadIdx.x; idx < S * S; idx += blockDim.x) {
    const int i = idx / S, j = idx % S;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += q[i * Dp + d] * k[j * Dp + d];
    P[i * Sp + j] = s * a.scale;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int i = wave; i < S; i += nw) {
    const float x = lane < S ? P[i * Sp + lane] : -INFINITY;
    const float m = wave_max(x);
    const float e = lane < S ? __expf(x - m) : 0.f;
    const float sum = wave_sum(e);
    if (lane < S) P[i * Sp + lane] = e / sum;
    if (lane == 0) a.lse[((size_t)b * a.Hl + h) * S + i] = m + __logf(sum);
  }
  __syncthreads();
  uint16_t* obase = a.o + (size_t)b * S * a.ld_o + h * D;
  // pooled output (mean over the S rows) for the pooled row-parallel fc_o; with
  // blockDim % D == 0 each thread keeps one column, so it sums in registers
  float* colsum = q;  // q is dead after the scores
  const bool pool = a.pool != nullptr;
  if (pool) {
    for (int c = threadIdx.x; c < D; c += blockDim.x) colsum[c] = 0.f;
    __syncthreads();
  }
  const bool fixed_col = (blockDim.x % D) == 0;
  float ps = 0.f;
  for (int idx = threadIdx.x; idx < S * D; idx += blockDim.x) {
    const int i = idx / D, d = idx % D;
    float acc = 0.f;
    for (int j = 0; j < S; ++j) acc += P[i * Sp + j] * v[j * Dp + d];
    st_bf16(obase + (size_t)i * a.ld_o + d, acc);
    if (pool) {
      if (fixed_col) ps += acc;
      else atomicAdd(&colsum[d], acc);
    }
  }
  if (pool) {
    if (fixed_col && threadIdx.x < S * D) atomicAdd(&colsum[threadIdx.x % D], ps);
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += blockDim.x)
      st_bf16(a.pool + (size_t)b * a.ld_pool + h * D + d, colsum[d] / (float)S);
  }
}

__global__ void __launch_bounds__(256) k_attn_bwd(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int S = a.S, D = a.D, Dp = D + 1, Sp = S + 1;
  const int b = blockIdx.x / a.Hl, h = blockIdx.x % a.Hl;
  float* q = sm;
  float* k = q + S * Dp;
  float* v = k + S * Dp;
  float* o = v + S * Dp;
  float* dO = o + S * Dp;
  float* P = dO + S * Dp;
  float* dS = P + S * Sp;
  float* delta = dS + S * Sp;
  const int HD = a.Hl * D;
  const uint16_t* base = a.qkv + (size_t)b * S * a.ld_qkv + h * D;
  stage(q, base, S, D, a.ld_qkv);
  stage(k, base + HD, S, D, a.ld_qkv);
  stage(v, base + 2 * HD, S, D, a.ld_qkv);
  stage(o, a.o + (size_t)b * S * a.ld_o + h * D, S, D, a.ld_o);
  {  // dO rows may be a broadcast of one pooled-gradient row (rstride 0)
    const uint16_t* db = a.dout + (size_t)b * a.dout_bstride + h * D;
    if (a.dout_rstride == 0) {
      stage(dO, db, 1, D, 0);
      __syncthreads();
      for (int idx = threadIdx.x; idx < (S - 1) * D; idx += blockDim.x) {
        const int i = 1 + idx / D, d = idx % D;
        dO[i * Dp + d] = dO[d];
      }
    } else {
      stage(dO, db, S, D, a.dout_rstride);
    }
  }
  __syncthreads();
  const float* lse = a.lse + ((size_t)b * a.Hl + h) * S;
  for (int idx = threadIdx.x; idx < S * S; idx += blockDim.x) {
    const int i = idx / S, j = idx % S;
    float s = 0.f, dp = 0.f;
    for (int d = 0; d < D; ++d) {
      s += q[i * Dp + d] * k[j * Dp + d];
      dp += dO[i * Dp + d] * v[j * Dp + d];
    }
    P[i * Sp + j] = __expf(s * a.scale - lse[i]);
    dS[i * Sp + j] = dp;
  }
  for (int i = threadIdx.x; i < S; i += blockDim.x) {
    float t = 0.f;
    for (int d = 0; d < D; ++d) t += dO[i * Dp + d] * o[i * Dp + d];
    delta[i] = t;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < S * S; idx += blockDim.x) {
    const int i = idx / S, j = idx % S;
    dS[i * Sp + j] = P[i * Sp + j] * (dS[i * Sp + j] - delta[i]);
  }
  __syncthreads();
  uint16_t* gq = a.dqkv + (size_t)b * S * a.ld_qkv + h * D;
  uint16_t* gk = gq + HD;
  uint16_t* gv = gq + 2 * HD;
  float* colsum = delta + S;  // 3*D floats: per-block column sums for the QKV bias gradient
  for (int c = threadIdx.x; c < 3 * D; c += blockDim.x) colsum[c] = 0.f;
  __syncthreads();
  // when blockDim is a multiple of D every thread keeps one column d for all its
  // rows, so the bias column sums accumulate in registers (one LDS atomic per thread)
  const bool fixed_col = (blockDim.x % D) == 0;
  float sq = 0.f, sk = 0.f, sv = 0.f;
  for (int idx = threadIdx.x; idx < S * D; idx += blockDim.x) {
    const int i = idx / D, d = idx % D;  // i: query row for dQ, key row for dK / dV
    float dq = 0.f, dk = 0.f, dv = 0.f;
    for (int j = 0; j < S; ++j) {
      dq += dS[i * Sp + j] * k[j * Dp + d];
      dk += dS[j * Sp + i] * q[j * Dp + d];
      dv += P[j * Sp + i] * dO[j * Dp + d];
    }
    dq *= a.scale;
    dk *= a.scale;
    st_bf16(gq + (size_t)i * a.ld_qkv + d, dq);
    st_bf16(gk + (size_t)i * a.ld_qkv + d, dk);
    st_bf16(gv + (size_t)i * a.ld_qkv + d, dv);
    if (a.dbias) {
      if (fixed_col) {
        sq += dq; sk += dk; sv += dv;
      } else {
        atomicAdd(&colsum[d], dq);
        atomicAdd(&colsum[D + d], dk);
        atomicAdd(&colsum[2 * D + d], dv);
      }
    }
  }
  if (a.dbias && fixed_col && threadIdx.x < S * D) {
    const int d = threadIdx.x % D;
    atomicAdd(&colsum[d], sq);
    atomicAdd(&colsum[D + d], sk);
    atomicAdd(&colsum[2 * D + d], sv);
  }
  if (a.dbias) {
    __syncthreads();
    for (int c = threadIdx.x; c < 3 * D; c += blockDim.x) {
      const int part = c / D, d = c % D;
      atomicAdd(a.dbias + part * HD + h * D + d, colsum[c]);
    }
  }
}

size_t fwd_lds(int S, int D) { return sizeof(float) * (3 * S * (D + 1) + S * (S + 1)); }
size_t bwd_lds(int S, int D) { return sizeof(float) * (5 * S * (D + 1) + 2 * S * (S + 1) + S + 3 * D); }

void check_dims(int S, int D, bool bwd) {
  if (S < 1 || S > 64 || D < 1 || D > 256) throw std::invalid_argument("attn_small: need 1 <= S <= 64, D <= 256");
  if ((bwd ? bwd_lds(S, D) : fwd_lds(S, D)) > 160 * 1024) throw std::invalid_argument("attn_small: tile exceeds LDS");
}

// Fused pooled fc_o (fwd: logits from the pooled attention output; bwd: the
// pooled output's gradient from dZ) needs the MFMA kernels' workgroup layout.
static void check_fused_fc(const AttnArgs& a, bool bwd) {
  if (!attn::mfma_supported(a, bwd) || a.n_out < 1 || a.n_out > 16 || 4 % a.Hl || !a.wo)
    throw std::invalid_argument("attention: fused fc_o needs S <= 16, D in {32, 64, 128}, Hl | 4, n_out <= 16");
  if (bwd && (a.ld_dz < 16 || a.ld_dz % 8 || ((uint64_t)a.dz % 16)))
    throw std::invalid_argument("attention: fused fc_o backward needs dz rows of >= 16 bf16, 16-B aligned");
  if (!bwd && !a.pool) throw std::invalid_argument("attention: fused fc_o forward needs the pooled output");
}

void attn_fwd(uint64_t qkv, uint64_t o, uint64_t lse, int B, int S, int Hl, int D, int ld_qkv, int ld_o, float scale,
              uint64_t pool, int ld_pool, uint64_t stream, uint64_t wo, int ld_wo, int n_out, uint64_t zp, int ld_zp,
              uint64_t bo, uint64_t ztok, int ld_zt, int zrows, const std::vector<uint64_t>& zpush) {
  check_dims(S, D, false);
  AttnArgs a{(const uint16_t*)qkv, (uint16_t*)o, (float*)lse, nullptr, nullptr, nullptr, B, S, Hl, D, ld_qkv, ld_o, scale,
             (uint16_t*)pool, ld_pool, 0, 0, (const uint16_t*)wo, ld_wo, n_out, (float*)zp, ld_zp, (const float*)bo,
             nullptr, 0, 1.0f};
  if (zp) check_fused_fc(a, false);
  if (ztok || zrows) {
    // per-token fused fc_o (local z, or pushed row blocks): the MFMA kernel's workgroup layout
    if (zp || !attn::mfma_supported(a, false) || n_out < 1 || n_out > 16 || 4 % Hl || !wo || ld_wo % 8 ||
        (wo % 16) || ld_zt < 16 || ld_zt % 4 || (ztok % 16))
      throw std::invalid_argument("attention: per-token fused fc_o needs S <= 16, D in {32, 64, 128}, Hl | 4, "
                                  "n_out <= 16, 16-B aligned W_o rows, z rows of >= 16 floats");
    if (zrows) {
      const int64_t M = (int64_t)B * S;
      const int64_t blocks = M / zrows;
      if (zrows % S || M % zrows || blocks < 1 || blocks > 16 || (int64_t)zpush.size() != blocks)
        throw std::invalid_argument("attention: push fc_o needs whole sequences per block (zrows % S == 0), "
                                    "B*S = blocks x zrows and one target per block (<= 16)");
      for (int64_t j = 0; j < blocks; ++j) {
        if (!zpush[j] || zpush[j] % 16) throw std::invalid_argument("attention: push fc_o targets must be 16-B aligned");
        a.zpush[j] = reinterpret_cast<float*>(zpush[j]);
      }
    }
    a.ztok = reinterpret_cast<float*>(ztok);
    a.ld_zt = ld_zt;
    a.zrows = zrows;
  }
  if (attn::mfma_supported(a, false)) {
    attn::launch_fwd_mfma(a, (hipStream_t)stream);
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(k_attn_fwd, dim3(B * Hl), dim3(256), fwd_lds(S, D), (hipStream_t)stream, a);
  CCMPI_HIP_CHECK(hipGetLastError());
}

// Fused QKV projection + attention + per-token fc_o (attn_mfma.hip k_qkv_attn16_fwd): the
// harness forward's QKV GEMM, attention and fc_o in one kernel (W_h held in registers).
void attn_qkv_fwd(uint64_t xq, int ld_xq, int kq, uint64_t wq, int ld_wq, uint64_t bq, uint64_t qkv_out, int ld_qkv,
                  uint64_t lse, int B, int S, int Hl, int D, float scale, uint64_t pool, int ld_pool, uint64_t wo,
                  int ld_wo, int n_out, uint64_t bo, uint64_t ztok, int ld_zt, int zrows,
                  const std::vector<uint64_t>& zpush, uint64_t stream, uint64_t img, uint64_t xq_out, uint64_t zmean,
                  int ld_zmean, uint64_t fold_wq, int ld_fold_wq, uint64_t fold_we, int ld_fold_we, uint64_t fold_out,
                  int ld_fold_out, int fold_R, int fold_d, uint64_t tstamp) {
  if (S < 1 || S > 16 || !(D == 32 || D == 64) || Hl < 1 || 4 % Hl || kq < 8 || kq > 72 || kq % 8 || ld_xq % 8 ||
      ld_wq % 8 || ld_wo % 8 || (xq % 16) || (wq % 16) || (wo % 16) || !wo || !bq || (bq % 16) || n_out < 1 ||
      n_out > 16 ||
      ld_zt < 16 || ld_zt % 4 || (ztok % 16) || (!ztok && !zrows && !zmean) || (qkv_out && (ld_qkv % 8 || qkv_out % 16)) ||
      (zmean && (zmean % 16 || ld_zmean % 4 || ld_zmean < 16 || zrows)) ||
      false)
    throw std::invalid_argument("attention: fused QKV forward needs S <= 16, D in {32, 64}, Hl | 4, kq % 8 == 0 and "
                                "<= 72 (the bias rides in two spare depth columns), 16-B aligned rows, n_out <= 16, "
                                "z rows of >= 16 floats (% 4), a z target");
  if (img && (S != 16 || kq < 66 || (img % 16) || (xq_out % 16)))
    throw std::invalid_argument("attention: fused patchify is the MNIST 28x28 / 7x7 case (S = 16, kq >= 66)");
  if (!img && (xq_out || !xq)) throw std::invalid_argument("attention: patch rows xq needed (xq_out only with img)");
  if (fold_out && (!img || !fold_wq || !fold_we || fold_R < 1 || fold_d < 4 || fold_d % 4 || fold_d > 16 * 4 * 16 ||
                   ld_fold_wq % 4 || ld_fold_wq < fold_d || ld_fold_we < kq || ld_fold_out < kq || (fold_wq % 16) ||
                   fold_out == wq))
    throw std::invalid_argument("attention: the fold tail needs image mode, fp32 Wq [R][d] (16-B aligned, d % 4 == 0, "
                                "d <= 1024) and We [d][kq], and an output other than the W_eff being read");
  AttnArgs a{};
  a.lse = (float*)lse;  // null: not stored (an inference forward: only a backward reads it)
  a.tstamp = (unsigned long long*)tstamp;
  a.B = B; a.S = S; a.Hl = Hl; a.D = D; a.ld_qkv = ld_qkv; a.scale = scale;
  a.pool = (uint16_t*)pool; a.ld_pool = ld_pool;
  a.wo = (const uint16_t*)wo; a.ld_wo = ld_wo; a.n_out = n_out; a.bo = (const float*)bo;
  a.xq = (const uint16_t*)xq; a.ld_xq = ld_xq; a.kq = kq;
  a.wq = (const uint16_t*)wq; a.ld_wq = ld_wq; a.bq = (const float*)bq; a.qkv_out = (uint16_t*)qkv_out;
  a.img = (const float*)img; a.xq_out = (uint16_t*)xq_out;
  a.zp = (float*)zmean; a.ld_zp = ld_zmean;  // mean over the tokens of z (the local form's logits)
  a.fold_wq = (const float*)fold_wq; a.ld_fold_wq = ld_fold_wq; a.fold_we = (const float*)fold_we;
  a.ld_fold_we = ld_fold_we; a.fold_out = (uint16_t*)fold_out; a.ld_fold_out = ld_fold_out;
  a.fold_R = fold_R; a.fold_d = fold_d; a.fold_kp = kq;
  static const int at_start = std::getenv("CCMPI_FOLD_TAIL_AT") && std::string(std::getenv("CCMPI_FOLD_TAIL_AT")) == "end" ? 0 : 1;
  a.fold_at_start = at_start;
  a.ztok = (float*)ztok; a.ld_zt = ld_zt; a.zrows = zrows;
  if (zrows) {
    const int64_t M = (int64_t)B * S;
    const int64_t blocks = M / zrows;
    if (zrows % S || M % zrows || blocks < 1 || blocks > 16 || (int64_t)zpush.size() != blocks)
      throw std::invalid_argument("attention: push fc_o needs whole sequences per block (zrows % S == 0), "
                                  "B*S = blocks x zrows and one target per block (<= 16)");
    for (int64_t j = 0; j < blocks; ++j) {
      if (!zpush[j] || zpush[j] % 16) throw std::invalid_argument("attention: push fc_o targets must be 16-B aligned");
      a.zpush[j] = reinterpret_cast<float*>(zpush[j]);
    }
  }
  if (B == 0) return;
  attn::launch_qkv_fwd_mfma(a, (hipStream_t)stream);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void attn_bwd(uint64_t qkv, uint64_t o, uint64_t lse, uint64_t dout, uint64_t dqkv, uint64_t dbias, int B, int S,
              int Hl, int D, int ld_qkv, int ld_o, float scale, int dout_bstride, int dout_rstride, uint64_t stream,
              uint64_t dz, int ld_dz, uint64_t wo, int ld_wo, int n_out, float dz_scale) {
  check_dims(S, D, true);
  AttnArgs a{(const uint16_t*)qkv, (uint16_t*)o, (float*)lse, (const uint16_t*)dout, (uint16_t*)dqkv, (float*)dbias,
             B, S, Hl, D, ld_qkv, ld_o, scale, nullptr, 0, dout_bstride, dout_rstride, (const uint16_t*)wo, ld_wo,
             n_out, nullptr, 0, nullptr, (const uint16_t*)dz, ld_dz, dz_scale};
  if (dz) check_fused_fc(a, true);
  if (attn::mfma_supported(a, true)) {
    attn::launch_bwd_mfma(a, (hipStream_t)stream);
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(k_attn_bwd, dim3(B * Hl), dim3(256), bwd_lds(S, D), (hipStream_t)stream, a);
  CCMPI_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Fused AdamW on a flat fp32 parameter buffer + bf16 compute copy (one pass).
// g is the (DP-summed) gradient; grad_scale folds the 1/dp average in.  Up to
// kMaxT regions of the flat buffer (row-major [rows][cols] weights) also get a
// TRANSPOSED bf16 copy ([cols][rows]), so backward GEMMs that need W^T read it
// directly instead of launching a transpose every step.
// ---------------------------------------------------------------------------
constexpr int kMaxT = 4, kTT = 32;  // transposed regions, transpose tile (32x32: enough workgroups to fill the chip)
struct TRegions {
  uint64_t off[kMaxT], rows[kMaxT], cols[kMaxT];
  uint16_t* dst[kMaxT];
  int tiles[kMaxT + 1];  // prefix sums of 64x64 tiles per region
  int n;
};

__device__ __forceinline__ bool in_regions(const TRegions& tr, uint64_t i) {
  for (int k = 0; k < tr.n; ++k)
    if (i >= tr.off[k] && i - tr.off[k] < tr.rows[k] * tr.cols[k]) return true;
  return false;
}

struct AdamArgs {
  float* p;
  float* g;
  float* m;
  float* v;
  uint16_t* p16;
  uint64_t n;
  float lr, b1, b2, eps, wd, bc1, bc2, grad_scale;
  int zero_grad;
  // optional device step counter (a HIP-graph-captured or plan-replayed step): two slots of
  // "steps done" used alternately.  Every workgroup reads t = *step_dev + 1 and workgroup 0
  // writes t into the other slot (*step_next), which no workgroup of this launch reads; the
  // next step (the other recording of the pair) reads that slot.  So a replayed step applies
  // the right bias corrections with no host-side argument and no extra launch.  (A one-thread
  // advance kernel after this one cost 4-5 us per step; a last-workgroup ticket, 2000+
  // contended atomics on one address, 70 us.)
  int* step_dev;
  int* step_next;
};

// the bias corrections of step t = step_dev[0] + 1
__device__ __forceinline__ void adam_device_step(AdamArgs& a) {
  if (!a.step_dev) return;
  const int t = __hip_atomic_load(a.step_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.step_next[0] = t;
  a.bc1 = 1.f - powf(a.b1, (float)t);
  a.bc2 = 1.f - powf(a.b2, (float)t);
}

// one AdamW element update on already-loaded values; returns the new bf16 bits
__device__ __forceinline__ float adam_math(const AdamArgs& a, float pi, float gi, float& mi, float& vi) {
  gi *= a.grad_scale;
  mi = a.b1 * mi + (1.f - a.b1) * gi;
  vi = a.b2 * vi + (1.f - a.b2) * gi * gi;
  pi *= 1.f - a.lr * a.wd;
  return pi - a.lr * (mi / a.bc1) / (sqrtf(vi / a.bc2) + a.eps);
}

// Workgroups [0, flat) stride over the flat buffer, skipping the transposed
// regions; every further workgroup owns one 32x32 tile of a region: it updates
// the tile row-major (coalesced), stages the bf16 values in LDS and writes the
// transposed tile with coalesced rows.  All four state arrays are distinct
// (restrict), and a tile's 16 elements per thread are loaded before any store.
__global__ void __launch_bounds__(256) k_adamw(AdamArgs a, TRegions tr, int flat) {
  adam_device_step(a);
  float* __restrict__ P = a.p;
  float* __restrict__ Gr = a.g;
  float* __restrict__ Mo = a.m;
  float* __restrict__ Vo = a.v;
  uint16_t* __restrict__ P16 = a.p16;
  if ((int)blockIdx.x < flat) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)flat * blockDim.x) {
      if (tr.n && in_regions(tr, i)) continue;
      float mi = Mo[i], vi = Vo[i];
      const float pi = adam_math(a, P[i], Gr[i], mi, vi);
      if (a.zero_grad) Gr[i] = 0.f;
      Mo[i] = mi;
      Vo[i] = vi;
      P[i] = pi;
      if (P16) P16[i] = (uint16_t)f32_to_bf16_bits(pi);
    }
    return;
  }
  __shared__ uint16_t tile[kTT][kTT + 1];
  const int t = (int)blockIdx.x - flat;
  int k = 0;
  while (k + 1 < tr.n && t >= tr.tiles[k + 1]) ++k;
  const int R = (int)tr.rows[k], Cc = (int)tr.cols[k];
  const int ntc = (Cc + kTT - 1) / kTT, lt = t - tr.tiles[k];
  const int r0 = (lt / ntc) * kTT, c0 = (lt % ntc) * kTT;
  const int tx = threadIdx.x & (kTT - 1), ty = threadIdx.x / kTT;
  constexpr int RS = 256 / kTT;  // rows per pass
  constexpr int J = kTT / RS;
  float pv[J], gv[J], mv[J], vv[J];
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int r = r0 + ty + RS * jj, c = c0 + tx;
    const uint64_t i = tr.off[k] + (uint64_t)r * Cc + c;
    const bool ok = r < R && c < Cc;
    pv[jj] = ok ? P[i] : 0.f;
    gv[jj] = ok ? Gr[i] : 0.f;
    mv[jj] = ok ? Mo[i] : 0.f;
    vv[jj] = ok ? Vo[i] : 0.f;
  }
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int r = r0 + ty + RS * jj, c = c0 + tx;
    if (r < R && c < Cc) {
      const uint64_t i = tr.off[k] + (uint64_t)r * Cc + c;
      const float pi = adam_math(a, pv[jj], gv[jj], mv[jj], vv[jj]);
      if (a.zero_grad) Gr[i] = 0.f;
      Mo[i] = mv[jj];
      Vo[i] = vv[jj];
      P[i] = pi;
      const uint16_t h = (uint16_t)f32_to_bf16_bits(pi);
      if (P16) P16[i] = h;
      tile[ty + RS * jj][tx] = h;
    }
  }
  __syncthreads();
  for (int j = ty; j < kTT; j += RS) {  // dst[c][r]: consecutive tx -> consecutive r
    const int c = c0 + j, r = r0 + tx;
    if (r < R && c < Cc) tr.dst[k][(uint64_t)c * R + r] = tile[tx][j];
  }
}

// MNIST patchify: x[B][img*img] fp32 -> xp[B*S][kp] bf16 with, per token row,
// the patch pixels (p*p), a constant 1 (folds the embedding bias into the
// GEMM) and a one-hot position (folds the learned position embedding into the
// GEMM), zero-padded to kp.  One thread per 8-column chunk of a token row
// (one 16-B store); kp % 8 == 0.  Rows are ldo elements apart (ldo >= kp), so
// the patches can be written as the right-hand column block of a wider
// activation buffer ([h | xp], models/mnist_tp.py).
// IMG / P > 0: compile-time image and patch size (the MNIST 28 / 7 case), so every
// index division is a multiply-shift; 0 = runtime sizes.  32-bit indices (the
// 64-bit div/mod chain dominated the kernel: 6.8 us for 4.7 MB out).
template <int IMG, int P>
__global__ void __launch_bounds__(256) k_patchify(const float* __restrict__ x, uint16_t* __restrict__ xp, int B, int img_rt,
                                                  int p_rt, int kp, int ldo) {
  const int img = IMG > 0 ? IMG : img_rt, p = P > 0 ? P : p_rt;
  const int g = img / p, S = g * g, pp = p * p, nch = kp / 8;
  const unsigned total = (unsigned)B * S * nch;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int ch = (int)(e % nch);
    const unsigned row = e / nch;
    const int s = (int)(row % S);
    const float* xb = x + (size_t)(row / S) * img * img + (s / g) * p * img + (s % g) * p;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = ch * 8 + 2 * q + h;
        float v = 0.f;
        if (c < pp) v = xb[(c / p) * img + c % p];
        else if (c == pp || c == pp + 1 + s) v = 1.f;
        v2[h] = v;
      }
      w[q] = pk_bf16(v2[0], v2[1]);
    }
    *reinterpret_cast<uint4*>(xp + (size_t)row * ldo + ch * 8) = uint4{w[0], w[1], w[2], w[3]};
  }
}

void patchify(uint64_t x, uint64_t xp, int B, int img, int p, int kp, uint64_t stream, int ldo) {
  const int S = (img / p) * (img / p);
  if (ldo <= 0) ldo = kp;
  if (kp < p * p + 1 + S) throw std::invalid_argument("patchify: kp too small for pixels + bias + position columns");
  if (kp % 8 || ldo % 8 || ldo < kp || xp % 16)
    throw std::invalid_argument("patchify: kp % 8 == 0, ldo % 8 == 0, ldo >= kp and a 16-B aligned output required");
  const uint64_t total = (uint64_t)B * S * (kp / 8);
  if (total >= (1ull << 31)) throw std::invalid_argument("patchify: batch too large for 32-bit indexing");
  const int grid = (int)std::min<uint64_t>((total + 255) / 256, 8192);
  // (an LDS-staged variant -- whole images loaded with 16-B loads, rows built from
  // LDS -- measured 6.85 us against 5.8 us for this gather form)
  if (img == 28 && p == 7)
    hipLaunchKernelGGL((k_patchify<28, 7>), dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)x, (uint16_t*)xp,
                       B, img, p, kp, ldo);
  else
    hipLaunchKernelGGL((k_patchify<0, 0>), dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)x, (uint16_t*)xp,
                       B, img, p, kp, ldo);
  CCMPI_HIP_CHECK(hipGetLastError());
}

// Mean over each group of S consecutive fp32 rows (the per-token fc_o's logits: z rows ->
// one row per sequence), one thread per (group, 4 columns), rows summed in order -- the
// summation order of DeviceComm::inbox_mean, so the "plain" TP form (all-reduce of z, then
// this) and the "push" form (inbox_mean) give bitwise the same logits.
__global__ void __launch_bounds__(256) k_rows_mean(const float* __restrict__ z, int ld_z, float* __restrict__ out,
                                                   int ld_out, int groups, int S, int ncol4) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= groups * ncol4) return;
  const int gi = idx / ncol4, q = idx % ncol4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < S; ++i) {
    const float4 v = *reinterpret_cast<const float4*>(z + (size_t)(gi * S + i) * ld_z + 4 * q);
    acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
  }
  const float n = (float)S;
  *reinterpret_cast<float4*>(out + (size_t)gi * ld_out + 4 * q) = float4{acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n};
}

void rows_mean(uint64_t z, int ld_z, uint64_t out, int ld_out, int groups, int S, int ncol, uint64_t stream) {
  if (groups < 0 || S < 1 || ncol % 4 || ld_z % 4 || ld_out % 4 || z % 16 || out % 16 || ncol > ld_z || ncol > ld_out)
    throw std::invalid_argument("rows_mean: fp32 rows, ncol % 4 == 0, 16-B aligned rows");
  if (groups == 0) return;
  const int n = groups * (ncol / 4);
  hipLaunchKernelGGL(k_rows_mean, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const float*)z, ld_z,
                     (float*)out, ld_out, groups, S, ncol / 4);
  CCMPI_HIP_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_cast_bf16(const float* __restrict__ x, uint16_t* __restrict__ y, uint64_t n,
                                                   TRegions tr) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint16_t h = (uint16_t)f32_to_bf16_bits(x[i]);
    y[i] = h;
    for (int k = 0; k < tr.n; ++k) {  // (initialization path only: scattered writes are fine here)
      const uint64_t rel = i - tr.off[k];
      if (i >= tr.off[k] && rel < tr.rows[k] * tr.cols[k])
        tr.dst[k][(rel % tr.cols[k]) * tr.rows[k] + rel / tr.cols[k]] = h;
    }
  }
}

TRegions make_tregions(const std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t>>& regs) {
  if (regs.size() > (size_t)kMaxT) throw std::invalid_argument("at most 4 transposed regions");
  TRegions tr{};
  tr.n = (int)regs.size();
  tr.tiles[0] = 0;
  for (int k = 0; k < tr.n; ++k) {
    tr.off[k] = std::get<0>(regs[k]);
    tr.rows[k] = std::get<1>(regs[k]);
    tr.cols[k] = std::get<2>(regs[k]);
    tr.dst[k] = reinterpret_cast<uint16_t*>(std::get<3>(regs[k]));
    tr.tiles[k + 1] = tr.tiles[k] + (int)(((tr.rows[k] + kTT - 1) / kTT) * ((tr.cols[k] + kTT - 1) / kTT));
  }
  return tr;
}

void adamw(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t p16, uint64_t n, float lr, float b1, float b2,
           float eps, float wd, int step, float grad_scale, uint64_t stream,
           const std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t>>& tregions, bool zero_grad,
           uint64_t step_dev, int step_parity) {
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  const int flat = (int)std::min<uint64_t>((n + 255) / 256, 2048);
  const TRegions tr = make_tregions(tregions);
  if (step_dev % 8) throw std::invalid_argument("adamw: the device step counter must be 8-B aligned");
  if (step_parity != 0 && step_parity != 1) throw std::invalid_argument("adamw: step_parity must be 0 or 1");
  int* slots = reinterpret_cast<int*>(step_dev);
  AdamArgs a{(float*)p, (float*)g, (float*)m, (float*)v, (uint16_t*)p16, n, lr, b1, b2, eps, wd, bc1, bc2, grad_scale,
             zero_grad ? 1 : 0, slots ? slots + step_parity : nullptr, slots ? slots + (step_parity ^ 1) : nullptr};
  // (a float4-per-thread variant measured 7.8 vs 8.0 us at 650k parameters: not kept)
  hipLaunchKernelGGL(k_adamw, dim3(flat + tr.tiles[tr.n]), dim3(256), 0, (hipStream_t)stream, a, tr, flat);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void cast_bf16(uint64_t x, uint64_t y, uint64_t n, uint64_t stream,
               const std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t>>& tregions) {
  const int grid = (int)std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_cast_bf16, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)x, (uint16_t*)y, n,
                     make_tregions(tregions));
  CCMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void register_attn_ops(pybind11::module_& m) {
  m.def("rows_mean", &rows_mean, "out[g] = mean of fp32 rows z[g S .. g S + S) (ordered sum)", pybind11::arg("z"),
        pybind11::arg("ld_z"), pybind11::arg("out"), pybind11::arg("ld_out"), pybind11::arg("groups"),
        pybind11::arg("S"), pybind11::arg("ncol"), pybind11::arg("stream"),
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("attn_set_qkv_grid", [](int cap) { attn::g_qkv_grid_cap = cap > 0 ? cap : 256; },
        "workgroups of the fused QKV forward (default 256: one 8-wave workgroup per CU)", pybind11::arg("cap"));
  m.def("attn_set_qkv_fold_sched", [](int v) { attn::g_qkv_fold_sched = v < 0 ? -1 : (v ? 1 : 0); },
        "fused QKV forward with the in-kernel fold: 1 = fold owners take fewer pair blocks, 0 = grid-stride, "
        "-1 = CCMPI_QKV_FOLD_SCHED (default 1)", pybind11::arg("v"));
  m.def("attn_set_qkv_fold_grid", [](int v) { attn::g_qkv_fold_grid = v ? 1 : 0; },
        "fused QKV forward with the in-kernel fold: 1 = at small batches the grid grows by the fold's tiles "
        "(fold-only workgroups beside the attention ones), 0 = not (ranks sharing one GPU)", pybind11::arg("v"));
  m.def("attn_set_bwd_grid", [](int cap) { attn::g_bwd_grid_cap = cap > 0 ? cap : 0; },
        "backward kernel grid cap (tuning)");
  namespace py = pybind11;
  m.def("attn_small_fwd", &attn_fwd, py::arg("qkv"), py::arg("o"), py::arg("lse"), py::arg("B"), py::arg("S"),
        py::arg("Hl"), py::arg("D"), py::arg("ld_qkv"), py::arg("ld_o"), py::arg("scale"), py::arg("pool"),
        py::arg("ld_pool"), py::arg("stream"), py::arg("wo") = 0, py::arg("ld_wo") = 0, py::arg("n_out") = 0,
        py::arg("zp") = 0, py::arg("ld_zp") = 0, py::arg("bo") = 0, py::arg("ztok") = 0, py::arg("ld_zt") = 16,
        py::arg("zrows") = 0, py::arg("zpush") = std::vector<uint64_t>{}, py::call_guard<py::gil_scoped_release>());
  m.def("attn_qkv_fwd", &attn_qkv_fwd, py::arg("xq"), py::arg("ld_xq"), py::arg("kq"), py::arg("wq"), py::arg("ld_wq"),
        py::arg("bq"), py::arg("qkv_out"), py::arg("ld_qkv"), py::arg("lse"), py::arg("B"), py::arg("S"), py::arg("Hl"),
        py::arg("D"), py::arg("scale"), py::arg("pool"), py::arg("ld_pool"), py::arg("wo"), py::arg("ld_wo"),
        py::arg("n_out"), py::arg("bo"), py::arg("ztok"), py::arg("ld_zt"), py::arg("zrows"), py::arg("zpush"),
        py::arg("stream"), py::arg("img") = 0, py::arg("xq_out") = 0, py::arg("zmean") = 0, py::arg("ld_zmean") = 16,
        py::arg("fold_wq") = 0, py::arg("ld_fold_wq") = 0, py::arg("fold_we") = 0, py::arg("ld_fold_we") = 0,
        py::arg("fold_out") = 0, py::arg("ld_fold_out") = 0, py::arg("fold_R") = 0, py::arg("fold_d") = 0,
        py::arg("tstamp") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("attn_small_bwd", &attn_bwd, py::arg("qkv"), py::arg("o"), py::arg("lse"), py::arg("dout"), py::arg("dqkv"),
        py::arg("dbias"), py::arg("B"), py::arg("S"), py::arg("Hl"), py::arg("D"), py::arg("ld_qkv"), py::arg("ld_o"),
        py::arg("scale"), py::arg("dout_bstride"), py::arg("dout_rstride"), py::arg("stream"), py::arg("dz") = 0,
        py::arg("ld_dz") = 0, py::arg("wo") = 0, py::arg("ld_wo") = 0, py::arg("n_out") = 0,
        py::arg("dz_scale") = 1.0f, py::call_guard<py::gil_scoped_release>());
  m.def("adamw_step", &adamw, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("p16"), py::arg("n"),
        py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("step"),
        py::arg("grad_scale"), py::arg("stream"),
        py::arg("tregions") = std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t>>{},
        py::arg("zero_grad") = false, py::arg("step_dev") = 0, py::arg("step_parity") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("cast_bf16", &cast_bf16, py::arg("x"), py::arg("y"), py::arg("n"), py::arg("stream"),
        py::arg("tregions") = std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t>>{},
        py::call_guard<py::gil_scoped_release>());
  m.def("patchify", &patchify, py::arg("x"), py::arg("xp"), py::arg("B"), py::arg("img"), py::arg("p"), py::arg("kp"),
        py::arg("stream"), py::arg("ldo") = 0, py::call_guard<py::gil_scoped_release>());
}

}  // namespace dev
}  // namespace ccmpi
