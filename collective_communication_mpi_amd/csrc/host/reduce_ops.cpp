// Element-wise reduction kernels for the host plane (CPU buffers).
// Replaces np.add/np.minimum/np.maximum(..., out=) at reference
// mpi_wrapper/comm.py:89-93 and the library reductions behind MPI.Allreduce.
#include <complex>
#include <cstring>
#include <stdexcept>
#include <string>

#include "shm_comm.hpp"

namespace ccmpi {

namespace {

inline float half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t mant = h & 0x3ff;
  uint32_t bits;
  if (exp == 0) {
    if (mant == 0) {
      bits = sign;
    } else {  // subnormal: normalise
      int e = -1;
      do { ++e; mant <<= 1; } while ((mant & 0x400) == 0);
      mant &= 0x3ff;
      bits = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
    }
  } else if (exp == 0x1f) {
    bits = sign | 0x7f800000u | (mant << 13);
  } else {
    bits = sign | ((exp + 127 - 15) << 23) | (mant << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

inline uint16_t float_to_half(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  uint32_t sign = (x >> 16) & 0x8000;
  uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) {  // inf / nan
    return (uint16_t)(sign | 0x7c00 | (absx > 0x7f800000u ? 0x200 | ((absx >> 13) & 0x3ff) : 0));
  }
  if (absx >= 0x477ff000u) return (uint16_t)(sign | 0x7c00);  // overflow -> inf (RNE)
  if (absx < 0x38800000u) {  // subnormal or zero in half
    if (absx < 0x33000000u) return (uint16_t)sign;  // rounds to zero
    uint32_t e = absx >> 23;
    uint32_t m = (absx & 0x7fffff) | 0x800000;
    // value = m * 2^(e-150); half subnormal unit = 2^-24
    // result = round-nearest-even(m * 2^(e-126)) = RNE(m >> (126 - e))
    uint32_t sh = 126 - e;
    uint32_t q = m >> sh;
    uint32_t rem = m & ((1u << sh) - 1);
    uint32_t halfway = 1u << (sh - 1);
    if (rem > halfway || (rem == halfway && (q & 1))) ++q;
    return (uint16_t)(sign | q);
  }
  uint32_t e = (absx >> 23) - 127 + 15;
  uint32_t m = absx & 0x7fffff;
  uint32_t q = (e << 10) | (m >> 13);
  uint32_t rem = m & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (q & 1))) ++q;
  return (uint16_t)(sign | q);
}

inline float bf16_to_float(uint16_t h) {
  uint32_t bits = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

inline uint16_t float_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // keep NaN
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

template <typename T> struct OpSum  { static T f(T a, T b) { return a + b; } };
template <typename T> struct OpProd { static T f(T a, T b) { return a * b; } };
template <typename T> struct OpMin  { static T f(T a, T b) { return b < a ? b : a; } };
template <typename T> struct OpMax  { static T f(T a, T b) { return a < b ? b : a; } };
template <typename T> struct OpLand { static T f(T a, T b) { return (T)((a != T(0)) && (b != T(0))); } };
template <typename T> struct OpLor  { static T f(T a, T b) { return (T)((a != T(0)) || (b != T(0))); } };
template <typename T> struct OpLxor { static T f(T a, T b) { return (T)((a != T(0)) != (b != T(0))); } };
template <typename T> struct OpBand { static T f(T a, T b) { return (T)(a & b); } };
template <typename T> struct OpBor  { static T f(T a, T b) { return (T)(a | b); } };
template <typename T> struct OpBxor { static T f(T a, T b) { return (T)(a ^ b); } };
template <typename T> struct OpRepl { static T f(T, T b) { return b; } };

// NaN-propagating min/max for floats (numpy semantics: np.minimum propagates NaN).
template <typename T> struct FOpMin { static T f(T a, T b) { return (a != a) ? a : ((b != b) ? b : (b < a ? b : a)); } };
template <typename T> struct FOpMax { static T f(T a, T b) { return (a != a) ? a : ((b != b) ? b : (a < b ? b : a)); } };

template <typename T, template <typename> class OP>
void apply(void* dst, const void* src, size_t n) {
  T* d = static_cast<T*>(dst);
  const T* s = static_cast<const T*>(src);
  for (size_t i = 0; i < n; ++i) d[i] = OP<T>::f(d[i], s[i]);
}

template <template <typename> class OP, bool BF>
void apply16(void* dst, const void* src, size_t n) {
  uint16_t* d = static_cast<uint16_t*>(dst);
  const uint16_t* s = static_cast<const uint16_t*>(src);
  for (size_t i = 0; i < n; ++i) {
    float a = BF ? bf16_to_float(d[i]) : half_to_float(d[i]);
    float b = BF ? bf16_to_float(s[i]) : half_to_float(s[i]);
    float r = OP<float>::f(a, b);
    d[i] = BF ? float_to_bf16(r) : float_to_half(r);
  }
}

template <typename T>
bool int_dispatch(void* dst, const void* src, size_t n, int op) {
  switch (op) {
    case OP_SUM: apply<T, OpSum>(dst, src, n); return true;
    case OP_PROD: apply<T, OpProd>(dst, src, n); return true;
    case OP_MIN: apply<T, OpMin>(dst, src, n); return true;
    case OP_MAX: apply<T, OpMax>(dst, src, n); return true;
    case OP_LAND: apply<T, OpLand>(dst, src, n); return true;
    case OP_LOR: apply<T, OpLor>(dst, src, n); return true;
    case OP_LXOR: apply<T, OpLxor>(dst, src, n); return true;
    case OP_BAND: apply<T, OpBand>(dst, src, n); return true;
    case OP_BOR: apply<T, OpBor>(dst, src, n); return true;
    case OP_BXOR: apply<T, OpBxor>(dst, src, n); return true;
    case OP_REPLACE: apply<T, OpRepl>(dst, src, n); return true;
  }
  return false;
}

template <typename T>
bool float_dispatch(void* dst, const void* src, size_t n, int op) {
  switch (op) {
    case OP_SUM: apply<T, OpSum>(dst, src, n); return true;
    case OP_PROD: apply<T, OpProd>(dst, src, n); return true;
    case OP_MIN: apply<T, FOpMin>(dst, src, n); return true;
    case OP_MAX: apply<T, FOpMax>(dst, src, n); return true;
    case OP_LAND: apply<T, OpLand>(dst, src, n); return true;
    case OP_LOR: apply<T, OpLor>(dst, src, n); return true;
    case OP_LXOR: apply<T, OpLxor>(dst, src, n); return true;
    case OP_REPLACE: apply<T, OpRepl>(dst, src, n); return true;
  }
  return false;
}

template <bool BF>
bool half_dispatch(void* dst, const void* src, size_t n, int op) {
  switch (op) {
    case OP_SUM: apply16<OpSum, BF>(dst, src, n); return true;
    case OP_PROD: apply16<OpProd, BF>(dst, src, n); return true;
    case OP_MIN: apply16<FOpMin, BF>(dst, src, n); return true;
    case OP_MAX: apply16<FOpMax, BF>(dst, src, n); return true;
    case OP_REPLACE: apply<uint16_t, OpRepl>(dst, src, n); return true;
  }
  return false;
}

template <typename T>
bool complex_dispatch(void* dst, const void* src, size_t n, int op) {
  switch (op) {
    case OP_SUM: apply<std::complex<T>, OpSum>(dst, src, n); return true;
    case OP_PROD: apply<std::complex<T>, OpProd>(dst, src, n); return true;
    case OP_REPLACE: apply<std::complex<T>, OpRepl>(dst, src, n); return true;
  }
  return false;
}

bool dispatch(void* dst, const void* src, size_t n, int dt, int op) {
  switch (dt) {
    case DT_I8: return int_dispatch<int8_t>(dst, src, n, op);
    case DT_U8: case DT_BYTE: return int_dispatch<uint8_t>(dst, src, n, op);
    case DT_BOOL: {
      if (op == OP_SUM || op == OP_PROD || op == OP_MIN || op == OP_MAX) {
        // numpy bool semantics: sum->or, prod->and, min->and, max->or
        int mapped = (op == OP_SUM || op == OP_MAX) ? OP_LOR : OP_LAND;
        return int_dispatch<uint8_t>(dst, src, n, mapped);
      }
      return int_dispatch<uint8_t>(dst, src, n, op);
    }
    case DT_I16: return int_dispatch<int16_t>(dst, src, n, op);
    case DT_U16: return int_dispatch<uint16_t>(dst, src, n, op);
    case DT_I32: return int_dispatch<int32_t>(dst, src, n, op);
    case DT_U32: return int_dispatch<uint32_t>(dst, src, n, op);
    case DT_I64: return int_dispatch<int64_t>(dst, src, n, op);
    case DT_U64: return int_dispatch<uint64_t>(dst, src, n, op);
    case DT_F16: return half_dispatch<false>(dst, src, n, op);
    case DT_BF16: return half_dispatch<true>(dst, src, n, op);
    case DT_F32: return float_dispatch<float>(dst, src, n, op);
    case DT_F64: return float_dispatch<double>(dst, src, n, op);
    case DT_C64: return complex_dispatch<float>(dst, src, n, op);
    case DT_C128: return complex_dispatch<double>(dst, src, n, op);
  }
  return false;
}

}  // namespace

size_t dtype_size(int dt) {
  switch (dt) {
    case DT_I8: case DT_U8: case DT_BOOL: case DT_BYTE: return 1;
    case DT_I16: case DT_U16: case DT_F16: case DT_BF16: return 2;
    case DT_I32: case DT_U32: case DT_F32: return 4;
    case DT_I64: case DT_U64: case DT_F64: case DT_C64: return 8;
    case DT_C128: return 16;
  }
  throw std::invalid_argument("ccmpi: unknown dtype code " + std::to_string(dt));
}

bool reduce_supported(int dt, int op) {
  if (dt < 0 || dt >= DT_COUNT || op < 0 || op >= OP_COUNT) return false;
  char a[16] = {0}, b[16] = {0};
  return dispatch(a, b, 1, dt, op);
}

void reduce_inplace(void* dst, const void* src, size_t n, int dt, int op) {
  if (!dispatch(dst, src, n, dt, op))
    throw std::invalid_argument("ccmpi: reduction op " + std::to_string(op) +
                                " unsupported for dtype " + std::to_string(dt));
}

}  // namespace ccmpi
