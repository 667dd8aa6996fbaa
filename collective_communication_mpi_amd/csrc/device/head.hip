// Fused classifier head of the harness training step: softmax cross-entropy
// on z + b (z = pooled fc_o output, fp32 [B][ld_z], b = output bias), in one
// launch instead of ~9 PyTorch kernels (log_softmax, gather, sum, exp,
// index_put, div, column sum, zero + scatter of the bf16 gradient):
//
//   loss      += sum_b -log softmax(z_b + bias)[y_b] * scale
//   dz[b][c]   = (softmax(z_b + bias)[c] - [c == y_b]) * scale   (bf16, 0 for c >= n_classes)
//   dbias[c]  += sum_b dz[b][c]                                  (fp32)
//
// scale = 1 / global batch.  One thread per row (n_classes is small); the
// per-class bias gradient and the loss are reduced in LDS per workgroup and
// added with one atomic per class per workgroup.
#include <pybind11/pybind11.h>

#include "common.hpp"
#include "ops.hpp"

namespace ccmpi {
namespace dev {

namespace {

constexpr int kMaxClasses = 64;

__global__ void __launch_bounds__(64) k_xent_head(const float* __restrict__ z, int ld_z, const float* __restrict__ bias,
                                                   const void* __restrict__ y, int y64, int B, int C, int Cpad, float scale,
                                                   float* __restrict__ loss, uint16_t* __restrict__ dz, int ld_dz,
                                                   float* __restrict__ dbias) {
  __shared__ float s_db[kMaxClasses];
  __shared__ float s_loss;
  const int t = threadIdx.x;
  for (int c = t; c < C; c += blockDim.x) s_db[c] = 0.f;
  if (t == 0) s_loss = 0.f;
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + t;
  const bool live = b < B;  // every lane takes part in the wave reductions
  const float* zr = z + (size_t)(live ? b : 0) * ld_z;
  auto logit = [&](int c) { return zr[c] + (bias ? bias[c] : 0.f); };
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, logit(c));
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += __expf(logit(c) - m);
  const float inv = 1.f / s;
  const int label = !live ? -1 : y64 ? (int)reinterpret_cast<const int64_t*>(y)[b] : reinterpret_cast<const int32_t*>(y)[b];
  const float lse = m + __logf(s);
  const float zy = (label >= 0 && label < C) ? logit(label) : lse;
  auto wsum = [](float x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
  };
  const float l = wsum(live ? (lse - zy) * scale : 0.f);
  if ((t & 63) == 0) atomicAdd(&s_loss, l);
  uint16_t* dr = dz + (size_t)b * ld_dz;
  for (int c = 0; c < Cpad; ++c) {
    float g = 0.f;
    if (c < C) {
      g = live ? (__expf(logit(c) - m) * inv - (c == label ? 1.f : 0.f)) * scale : 0.f;
      const float gs = wsum(g);
      if ((t & 63) == 0) atomicAdd(&s_db[c], gs);
    }
    if (live) dr[c] = (uint16_t)f32_to_bf16_bits(g);
  }
  __syncthreads();
  if (dbias)
    for (int c = t; c < C; c += blockDim.x) atomicAdd(dbias + c, s_db[c]);
  if (t == 0) atomicAdd(loss, s_loss);
}


// Lane-per-class form (C <= Cpad <= 16): 16 lanes per row, 4 rows per wave,
// 16 rows per 256-thread workgroup.  max / sum over classes are 4-step
// shuffles, the dZ row is one contiguous 32-B store, and per-class column sums
// combine the 4 rows of a wave (xor 16, 32) before LDS and one atomic per
// class per workgroup.
__global__ void __launch_bounds__(256) k_xent_head16(const float* __restrict__ z, int ld_z,
                                                     const float* __restrict__ bias, const void* __restrict__ y, int y64,
                                                     int B, int C, int Cpad, float scale, float* __restrict__ loss,
                                                     uint16_t* __restrict__ dz, int ld_dz, float* __restrict__ dbias,
                                                     float* __restrict__ partial, unsigned* __restrict__ ticket) {
  __shared__ float s_db[4][16];
  __shared__ float s_loss[4];
  __shared__ bool s_last;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c = lane & 15;
  const int b = blockIdx.x * 16 + wave * 4 + (lane >> 4);
  const bool live = b < B;
  const float v = (live && c < C) ? z[(size_t)b * ld_z + c] + (bias ? bias[c] : 0.f) : -INFINITY;
  float m = v;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
  const float e = (c < C) ? __expf(v - m) : 0.f;
  float s = e;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o);
  const int label = !live ? -1 : y64 ? (int)reinterpret_cast<const int64_t*>(y)[b] : reinterpret_cast<const int32_t*>(y)[b];
  float l = (live && c == label) ? (m + __logf(s) - v) * scale : 0.f;
  const float gr = (live && c < C) ? (e / s - (c == label ? 1.f : 0.f)) * scale : 0.f;
  if (live && c < Cpad) dz[(size_t)b * ld_dz + c] = (uint16_t)f32_to_bf16_bits(gr);
  float cs = gr;
  cs += __shfl_xor(cs, 16);
  cs += __shfl_xor(cs, 32);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
  if (lane < 16) s_db[wave][lane] = cs;
  if (lane == 0) s_loss[wave] = l;
  __syncthreads();
  if (t < C && dbias) atomicAdd(dbias + t, s_db[0][t] + s_db[1][t] + s_db[2][t] + s_db[3][t]);
  // loss: per-workgroup partial, the last workgroup to finish sums them in a fixed
  // order and re-arms the ticket (no memset launch, deterministic sum)
  if (t == 0) {
    partial[blockIdx.x] = s_loss[0] + s_loss[1] + s_loss[2] + s_loss[3];
    __threadfence();
    s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && t < 64) {
    __threadfence();
    float acc = 0.f;
    for (int i = t; i < (int)gridDim.x; i += 64) acc += __hip_atomic_load(partial + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (t == 0) {
      *loss = acc;
      *ticket = 0u;
    }
  }
}

// Loss head + output-weight gradient in one launch, for the harness's pooled / per-token
// fc_o (logits z = pool W_o^T + o_b, pool = the sequence mean of the attention output):
// loss, dz (bf16) and dbias as k_xent_head16 (z already holds + o_b), and
//
//   dW_o[c][j] += sum_b dz[b][c] * pool[b][j]      (c < C, j < HD; bf16 dz and pool, fp32 sums)
//
// which the backward otherwise runs as a split-K TN GEMM dZ^T pool: a second launch of
// ~7 us at B = 2048 for 16 x 256 outputs.  Grid (ceil(B / 64), ceil(HD / 64)): workgroup
// (x, y) forms the gradient of rows 64x.. (every y recomputes that small softmax; y = 0
// alone stores dz, dbias and the loss partial; 4 lanes per row, 4 classes per lane), then the
// 16 x 64 dW_o tile of columns 64y..:
// wave q sums rows 16q..16q+15 for column 64y + lane from pool values fetched before the
// softmax, the four quarters meet in LDS, and one atomic per (class, column) leaves.
constexpr int kWoRows = 64;

__global__ void __launch_bounds__(256) k_xent_head_wo(const float* __restrict__ z, int ld_z, const void* __restrict__ y,
                                                      int y64, int B, int C, int Cpad, float scale,
                                                      float* __restrict__ loss, uint16_t* __restrict__ dz, int ld_dz,
                                                      float* __restrict__ dbias, const uint16_t* __restrict__ pool,
                                                      int ld_pool, int HD, float* __restrict__ dwo, int ld_dwo,
                                                      float* __restrict__ partial, unsigned* __restrict__ ticket) {
  __shared__ __attribute__((aligned(16))) float s_g[kWoRows][16];  // the rows' bf16-rounded gradient
  __shared__ float s_acc[3][16][64];  // row quarters 1..3 of the dW_o tile
  __shared__ float s_db[4][16];
  __shared__ float s_loss[4];
  __shared__ bool s_last;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int b0 = blockIdx.x * kWoRows;
  const bool head = blockIdx.y == 0;
  const int j = blockIdx.y * 64 + lane;
  uint16_t pv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int b = b0 + wave * 16 + r;
    pv[r] = (b < B && j < HD) ? pool[(size_t)b * ld_pool + j] : (uint16_t)0;
  }
  // softmax: 4 lanes per row (classes 4q .. 4q + 3 on lane q of the row), all 64 rows at once
  const int rl = t >> 2, q = t & 3, c0 = 4 * q;
  const int b = b0 + rl;
  const bool live = b < B;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (live && c0 + e < C) ? z[(size_t)b * ld_z + c0 + e] : -INFINITY;
  const int label = !live ? -1 : y64 ? (int)reinterpret_cast<const int64_t*>(y)[b] : reinterpret_cast<const int32_t*>(y)[b];
  float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  float ex[4], s = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ex[e] = (c0 + e < C) ? __expf(v[e] - m) : 0.f;
    s += ex[e];
  }
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  const float inv = 1.f / s, lse = m + __logf(s);
  float l = 0.f, gf[4];
  uint16_t gb[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + e;
    if (live && c == label) l += (lse - v[e]) * scale;
    const float gr = (live && c < C) ? (ex[e] * inv - (c == label ? 1.f : 0.f)) * scale : 0.f;
    gb[e] = (uint16_t)f32_to_bf16_bits(gr);
    gf[e] = gr;
  }
  *reinterpret_cast<float4*>(&s_g[rl][c0]) = float4{__uint_as_float((uint32_t)gb[0] << 16), __uint_as_float((uint32_t)gb[1] << 16),
                                                    __uint_as_float((uint32_t)gb[2] << 16), __uint_as_float((uint32_t)gb[3] << 16)};
  if (head && live) {
    if (c0 + 3 < Cpad) {
      *reinterpret_cast<uint2*>(dz + (size_t)b * ld_dz + c0) =
          uint2{(uint32_t)gb[0] | ((uint32_t)gb[1] << 16), (uint32_t)gb[2] | ((uint32_t)gb[3] << 16)};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c0 + e < Cpad) dz[(size_t)b * ld_dz + c0 + e] = gb[e];
    }
  }
  __syncthreads();
  float acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = __uint_as_float((uint32_t)pv[r] << 16);
    const float4* g = reinterpret_cast<const float4*>(s_g[wave * 16 + r]);
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      const float4 w = g[k4];
      acc[4 * k4 + 0] = fmaf(w.x, p, acc[4 * k4 + 0]);
      acc[4 * k4 + 1] = fmaf(w.y, p, acc[4 * k4 + 1]);
      acc[4 * k4 + 2] = fmaf(w.z, p, acc[4 * k4 + 2]);
      acc[4 * k4 + 3] = fmaf(w.w, p, acc[4 * k4 + 3]);
    }
  }
  if (wave > 0)
#pragma unroll
    for (int k = 0; k < 16; ++k) s_acc[wave - 1][k][lane] = acc[k];
  if (head) {
    // class sums over the wave's 16 rows (lanes with the same q), loss over the wave
    float cs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      cs[e] = gf[e];
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) cs[e] += __shfl_xor(cs[e], o);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
    if (lane < 4)
#pragma unroll
      for (int e = 0; e < 4; ++e) s_db[wave][4 * lane + e] = cs[e];
    if (lane == 0) s_loss[wave] = l;
  }
  __syncthreads();
  if (wave == 0 && j < HD) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < C)
        atomicAdd(dwo + (size_t)k * ld_dwo + j, acc[k] + s_acc[0][k][lane] + s_acc[1][k][lane] + s_acc[2][k][lane]);
  }
  if (head) {  // workgroup-uniform
    if (t < C && dbias) atomicAdd(dbias + t, s_db[0][t] + s_db[1][t] + s_db[2][t] + s_db[3][t]);
    // loss: the head workgroups' partials, summed in a fixed order by the last to finish
    if (t == 0) {
      partial[blockIdx.x] = s_loss[0] + s_loss[1] + s_loss[2] + s_loss[3];
      __threadfence();
      s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (s_last && t < 64) {
      __threadfence();
      float a = 0.f;
      for (int i = t; i < (int)gridDim.x; i += 64) a += __hip_atomic_load(partial + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
      if (t == 0) {
        *loss = a;
        *ticket = 0u;
      }
    }
  }
}

void xent_head_wo(uint64_t z, int ld_z, uint64_t y, bool y64, int B, int C, int Cpad, float scale, uint64_t loss,
                  uint64_t dz, int ld_dz, uint64_t dbias, uint64_t pool, int ld_pool, int HD, uint64_t dwo, int ld_dwo,
                  uint64_t stream, uint64_t workspace) {
  if (C < 1 || Cpad < C || Cpad > 16) throw std::invalid_argument("xent_head_wo: need 1 <= n_classes <= pad <= 16");
  if (!workspace || !pool || !dwo || HD <= 0 || ld_pool < HD || ld_dwo < HD)
    throw std::invalid_argument("xent_head_wo: workspace, pool [B][>= HD] and dW_o [C][>= HD] required");
  if (dz % 8 || ld_dz % 4) throw std::invalid_argument("xent_head_wo: dz 8-B aligned with a row stride % 4 == 0");
  if (B <= 0) return;
  hipLaunchKernelGGL(k_xent_head_wo, dim3((B + kWoRows - 1) / kWoRows, (HD + 63) / 64), dim3(256), 0,
                     (hipStream_t)stream, (const float*)z, ld_z, (const void*)y, y64 ? 1 : 0, B, C, Cpad, scale,
                     (float*)loss, (uint16_t*)dz, ld_dz, (float*)dbias, (const uint16_t*)pool, ld_pool, HD, (float*)dwo,
                     ld_dwo, reinterpret_cast<float*>(workspace) + 1, reinterpret_cast<unsigned*>(workspace));
  CCMPI_HIP_CHECK(hipGetLastError());
}

void xent_head(uint64_t z, int ld_z, uint64_t bias, uint64_t y, bool y64, int B, int C, int Cpad, float scale,
               uint64_t loss, uint64_t dz, int ld_dz, uint64_t dbias, uint64_t stream, uint64_t workspace) {
  if (C < 1 || C > kMaxClasses || Cpad < C) throw std::invalid_argument("xent_head: need 1 <= n_classes <= 64 <= pad");
  if (B <= 0) return;
  if (!(Cpad <= 16 && workspace))
    CCMPI_HIP_CHECK(hipMemsetAsync(reinterpret_cast<void*>(loss), 0, sizeof(float), (hipStream_t)stream));
  if (Cpad <= 16 && workspace) {
    // workspace: [0, 4) ticket (zero on first use, re-armed by the kernel), then one float per workgroup
    hipLaunchKernelGGL(k_xent_head16, dim3((B + 15) / 16), dim3(256), 0, (hipStream_t)stream, (const float*)z, ld_z,
                       (const float*)bias, (const void*)y, y64 ? 1 : 0, B, C, Cpad, scale, (float*)loss, (uint16_t*)dz,
                       ld_dz, (float*)dbias, reinterpret_cast<float*>(workspace) + 1,
                       reinterpret_cast<unsigned*>(workspace));
    CCMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  // one wave per workgroup: the kernel is latency bound, so spread rows over many CUs
  hipLaunchKernelGGL(k_xent_head, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, (const float*)z, ld_z,
                     (const float*)bias, (const void*)y, y64 ? 1 : 0, B, C, Cpad, scale, (float*)loss, (uint16_t*)dz, ld_dz,
                     (float*)dbias);
  CCMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void register_head_ops(pybind11::module_& m) {
  m.def("xent_head", &xent_head,
        "fused softmax cross-entropy head: loss (=), bf16 dz, dbias += column sums; workspace: 4 + 4*ceil(B/16) bytes, "
        "zero-initialized once (lane-per-class kernel), 0 = memset + atomics",
        pybind11::arg("z"), pybind11::arg("ld_z"), pybind11::arg("bias"), pybind11::arg("y"), pybind11::arg("y64"),
        pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("Cpad"), pybind11::arg("scale"), pybind11::arg("loss"),
        pybind11::arg("dz"), pybind11::arg("ld_dz"), pybind11::arg("dbias"), pybind11::arg("stream"),
        pybind11::arg("workspace") = 0, pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("xent_head_wo", &xent_head_wo,
        "xent_head (z already + bias, lane-per-class, workspace 4 + 4*ceil(B/64) bytes zeroed once) plus "
        "dW_o[c][j] += sum_b dz[b][c] pool[b][j] (bf16 pool, fp32 atomics) in one launch",
        pybind11::arg("z"), pybind11::arg("ld_z"), pybind11::arg("y"), pybind11::arg("y64"), pybind11::arg("B"),
        pybind11::arg("C"), pybind11::arg("Cpad"), pybind11::arg("scale"), pybind11::arg("loss"), pybind11::arg("dz"),
        pybind11::arg("ld_dz"), pybind11::arg("dbias"), pybind11::arg("pool"), pybind11::arg("ld_pool"),
        pybind11::arg("HD"), pybind11::arg("dwo"), pybind11::arg("ld_dwo"), pybind11::arg("stream"),
        pybind11::arg("workspace"), pybind11::call_guard<pybind11::gil_scoped_release>());
}

}  // namespace dev
}  // namespace ccmpi
