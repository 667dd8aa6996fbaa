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
}

}  // namespace dev
}  // namespace ccmpi
