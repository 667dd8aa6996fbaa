// Last-axis layout kernels for the tensor-parallel collects.
//
// reference model/func_impl.py:89-90,107-108 gathers (B,S,k) shards with an
// object all-gather and np.concatenate(axis=2); :182-186 splits grad_x along
// axis 2 (np.split) before an all-to-all + sum.  On device these become
//   interleave  : [p][M][k] -> [M][p*k]   (after a contiguous all-gather)
//   deinterleave: [M][p*k]  -> [p][M][k]  (before a block reduce-scatter)
// with M = B*S rows.  One 64-lane wave moves one k-row with 16-B vectors when
// the row is 16-B divisible, else 4-/2-/1-B units.
#include <pybind11/pybind11.h>

#include "common.hpp"
#include "ops.hpp"

namespace ccmpi {
namespace dev {

namespace {

template <typename U>
__global__ void __launch_bounds__(256) k_interleave(const char* __restrict__ src, char* __restrict__ dst,
                                                    uint64_t M, int p, uint64_t row_units, bool inverse) {
  // grid-stride over (m, j) row pairs; a wave per row
  const uint64_t rows = M * (uint64_t)p;
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t r = wave; r < rows; r += nwaves) {
    const uint64_t j = r / M, m = r % M;  // source block j, row m (contiguous reads)
    const U* s;
    U* d;
    if (!inverse) {
      s = reinterpret_cast<const U*>(src) + (j * M + m) * row_units;
      d = reinterpret_cast<U*>(dst) + (m * p + j) * row_units;
    } else {
      s = reinterpret_cast<const U*>(src) + (m * p + j) * row_units;
      d = reinterpret_cast<U*>(dst) + (j * M + m) * row_units;
    }
    for (uint64_t i = lane; i < row_units; i += 64) d[i] = s[i];
  }
}

void interleave(uint64_t src, uint64_t dst, uint64_t M, int p, uint64_t row_bytes, bool inverse, uint64_t stream) {
  if (M == 0 || row_bytes == 0 || p <= 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t rows = M * (uint64_t)p;
  const int grid = (int)std::min<uint64_t>((rows + 3) / 4, 4096);
  auto go = [&](auto unit) {
    using U = decltype(unit);
    hipLaunchKernelGGL((k_interleave<U>), dim3(grid), dim3(256), 0, st, (const char*)src, (char*)dst, M, p,
                       row_bytes / sizeof(U), inverse);
  };
  const uint64_t a = src | dst | row_bytes;
  if (a % 16 == 0) go(u32x4{});
  else if (a % 4 == 0) go(uint32_t{});
  else if (a % 2 == 0) go(uint16_t{});
  else go(uint8_t{});
  CCMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void register_layout_ops(pybind11::module_& m) {
  m.def("interleave_lastaxis", [](uint64_t src, uint64_t dst, uint64_t M, int p, uint64_t row_bytes, uint64_t stream) {
    interleave(src, dst, M, p, row_bytes, false, stream);
  }, "[p][M][k] -> [M][p*k] (bytes per k-row = row_bytes)");
  m.def("deinterleave_lastaxis", [](uint64_t src, uint64_t dst, uint64_t M, int p, uint64_t row_bytes, uint64_t stream) {
    interleave(src, dst, M, p, row_bytes, true, stream);
  }, "[M][p*k] -> [p][M][k]");
}

}  // namespace dev
}  // namespace ccmpi
