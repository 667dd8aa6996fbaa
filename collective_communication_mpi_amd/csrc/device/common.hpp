// Shared device-plane definitions: dtype/op codes (same numbering as the host
// plane, csrc/host/shm_comm.hpp), 16-byte vector helpers, element-wise
// reduction traits, and the cross-GPU signalling primitives used by every
// hand-written collective kernel.
//
// Memory-model notes (gfx950, 8 XCDs, private per-XCD L2, peers over xGMI):
//  * peer buffers are IPC-mapped coarse-grained HBM.  Every load of bytes a
//    peer produced in this launch, and every load of peer memory, is issued
//    system-coherent (`sc0 sc1`, aux = 17) so no L1/L2 copy can go stale across
//    calls; bytes we hand to peers are stored `sc0 sc1` (write-through) and
//    published by a system-scope release (`buffer_wbl2 sc0 sc1` + vmcnt(0))
//    before the flag.
//  * flags live in uncached signal buffers (hipDeviceMallocUncached) and are
//    written/polled with system-scope atomics; every spin is bounded by a
//    wall-clock budget (s_memrealtime, 100 MHz) and reports a timeout code
//    instead of hanging the GPU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

#define CCMPI_HIP_CHECK(expr)                                                              \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);     \
  } while (0)

namespace ccmpi {
namespace dev {

// dtype codes: identical to the host plane (csrc/host/shm_comm.hpp::DType)
enum DType : int {
  DT_I8 = 0, DT_U8, DT_I16, DT_U16, DT_I32, DT_U32, DT_I64, DT_U64,
  DT_F16, DT_BF16, DT_F32, DT_F64, DT_BOOL, DT_C64, DT_C128, DT_BYTE
};
enum ROp : int { OP_SUM = 0, OP_PROD, OP_MIN, OP_MAX };

constexpr int kMaxRanks = 16;     // ranks per device communicator
constexpr int kMaxSegs = 128;     // registered segments per rank: heap arenas + on-demand registrations (< 255)
constexpr int kMaxBlocks = 1024;  // max CTAs of one collective launch
constexpr int kCachePolicySys = 17;  // aux bits: sc0 | sc1 (system coherent)
// Stores of the collectives: sc0|sc1 write-through (aux 17), so bytes handed to a
// peer leave the XCD's L2 as they are produced instead of in one write-back burst
// at the release.  Measured against plain write-back stores (aux 0, compile with
// -DCCMPI_STORE_POLICY=0): identical TCC WRITE_SIZE and 0-9 % faster at 8 ranks
// (profiles/r2_coll/store_policy.md).  release_sys() is issued either way.
#ifndef CCMPI_STORE_POLICY
#define CCMPI_STORE_POLICY 17
#endif
constexpr int kStorePolicy = CCMPI_STORE_POLICY;
constexpr uint64_t kStepsPerEpoch = 64;  // > 2 * (kMaxRanks - 1) signals per call

inline size_t dtype_bytes(int dt) {
  switch (dt) {
    case DT_I8: case DT_U8: case DT_BOOL: case DT_BYTE: return 1;
    case DT_I16: case DT_U16: case DT_F16: case DT_BF16: return 2;
    case DT_I32: case DT_U32: case DT_F32: return 4;
    case DT_I64: case DT_U64: case DT_F64: case DT_C64: return 8;
    case DT_C128: return 16;
  }
  throw std::invalid_argument("ccmpi device: unknown dtype " + std::to_string(dt));
}

// ---------------------------------------------------------------------------
// device side tables
// ---------------------------------------------------------------------------
// Per-rank uncached signal buffer.  Peers write into OUR buffer at [..][their rank].
struct Signals {
  uint64_t flag[4][kMaxBlocks][kMaxRanks];  // phase x block x source rank
  uint64_t addr[2][kMaxBlocks][kMaxRanks];  // published (seg, offset) codes per block
  // step counters of the pipelined schedules (ring, recursive halving/doubling):
  // value = epoch * kStepsPerEpoch + step, so one monotonic word per (block, source)
  uint64_t step[kMaxBlocks][kMaxRanks];
  uint32_t error;                           // first timeout/ fault code seen
  uint32_t pad[15];
};

// Per-communicator table, resident in device memory, read by every kernel.
struct PeerTable {
  Signals* sig[kMaxRanks];               // sig[j]: rank j's signal buffer (mapped)
  char* seg[kMaxRanks][kMaxSegs];        // seg[j][s]: base of rank j's segment s
  uint64_t seg_bytes[kMaxSegs];
  char* ll[kMaxRanks];                    // ll[j]: rank j's LL buffer (uncached, mapped; null until set up)
  uint32_t* host_err;                    // pinned host word mirroring sig[rank]->error (watchdog)
  int rank;
  int size;
  int nsegs;
  int pad;
};

// Encodes "segment s, byte offset o" of a symmetric buffer.  Value 0 = none.
__host__ __device__ inline uint64_t addr_code(int seg, uint64_t off) {
  return ((uint64_t)(seg + 1) << 56) | (off & ((1ull << 56) - 1));
}
__device__ inline char* resolve(const PeerTable* pt, int peer, uint64_t code) {
  const int s = (int)(code >> 56) - 1;
  return pt->seg[peer][s] + (code & ((1ull << 56) - 1));
}

// ---------------------------------------------------------------------------
// memory helpers
// ---------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// 16-byte system-coherent load / store of an arbitrary (16-B aligned) address.
__device__ __forceinline__ u32x4 ld_sys16(const void* p) {
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 16, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, kCachePolicySys);
}
__device__ __forceinline__ void st_sys16(void* p, u32x4 v) {
  auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 16, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, 0, 0, kStorePolicy);
}
// Buffer-resource form: one descriptor per base, per-lane byte offsets (< 4 GiB).
struct Rsrc {
  __amdgpu_buffer_rsrc_t r;
};
__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return Rsrc{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000)};
}
__device__ __forceinline__ u32x4 ld16(Rsrc r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r.r, off, 0, kCachePolicySys);
}
__device__ __forceinline__ void st16(Rsrc r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r.r, off, 0, kStorePolicy);
}

// A pointer every lane holds identically, made provably wave-uniform (SGPRs), so
// buffer descriptors built from it need no waterfall loop.
__device__ __forceinline__ char* uniform_ptr(char* p) {
  uint64_t v = (uint64_t)p;
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (char*)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// Bounded wait until *p >= want (system scope). Returns false on timeout and
// records `code` in the local signal buffer's error word.
//
// Acquire side of the flag protocol.  The spin itself uses relaxed loads (a
// system-scope acquire load per iteration would invalidate the caches on
// every spin).  Once the flag is seen, a system-scope acquire fence orders
// every later load of this wave after the flag load and invalidates this
// CU's vector L1 / the XCD's L2 lines that could hold stale copies of peer
// data (gfx950: `buffer_inv sc0 sc1`).  The waiting lanes then reach
// __syncthreads() before any other wave of the workgroup touches peer data;
// the barrier orders those waves after the fence, and their loads are issued
// system-coherent (sc0 sc1) as well, so they never hit a line the fence did
// not cover.  The release side is `release_sys()` + the flag store: every
// store of the workgroup has completed into its XCD's L2 (vmcnt(0) before the
// barrier), `buffer_wbl2 sc0 sc1` writes that L2's dirty lines (this kernel's
// and any earlier kernel's) back to memory, and vmcnt(0) orders the flag
// store after the write-back.
__device__ __forceinline__ bool wait_geq(const uint64_t* p, uint64_t want, uint64_t budget_ticks,
                                         uint32_t* err, uint32_t code) {
  uint64_t t0 = 0;
  uint32_t spins = 0;
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if ((++spins & 63) == 0) {
      uint64_t t = now_ticks();
      if (t0 == 0) t0 = t;
      else if (t - t0 > budget_ticks) {
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}

// Mirror a timeout code into the host-mapped watchdog word (no device sync needed to see it).
__device__ __forceinline__ void report_host(const PeerTable* pt, uint32_t code) {
  if (pt->host_err) __hip_atomic_store(pt->host_err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void signal_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void release_sys() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void acquire_sys() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// element-wise reduction on 16-byte vectors
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
// fp32 -> bf16 bits, round to nearest even, NaN stays NaN: gfx950's v_cvt_pk_bf16_f32 (one
// VALU op; the integer RNE sequence it replaces compiled to an exec-mask branch per value for
// its NaN test).  Denormals are preserved (the kernels' fp32 denorm mode).
__device__ __forceinline__ uint32_t f32_to_bf16_bits(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
// two fp32 -> packed bf16 pair (lo = a): ONE v_cvt_pk_bf16_f32 (the scalar form above, OR-ed
// in pairs, compiles to two conversions + shift + or)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t{a, b}), b2_t));
}

template <int OP, typename A>
__device__ __forceinline__ A apply_op(A a, A b) {
  if constexpr (OP == OP_SUM) return a + b;
  else if constexpr (OP == OP_PROD) return a * b;
  else if constexpr (OP == OP_MIN) return b < a ? b : a;
  else return a < b ? b : a;
}

// Accumulator view of one 16-byte vector.
template <int DT> struct VecAcc;

template <> struct VecAcc<DT_F32> {
  static constexpr int N = 4;
  float v[4];
  __device__ __forceinline__ void load(u32x4 x) { for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(x[i]); }
  template <int OP> __device__ __forceinline__ void acc(u32x4 x) {
    for (int i = 0; i < 4; ++i) v[i] = apply_op<OP>(v[i], __uint_as_float(x[i]));
  }
  __device__ __forceinline__ u32x4 store() const {
    u32x4 r; for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(v[i]); return r;
  }
};

template <> struct VecAcc<DT_BF16> {
  static constexpr int N = 8;
  float v[8];
  __device__ __forceinline__ void load(u32x4 x) {
    for (int i = 0; i < 4; ++i) { v[2 * i] = bf16_lo(x[i]); v[2 * i + 1] = bf16_hi(x[i]); }
  }
  template <int OP> __device__ __forceinline__ void acc(u32x4 x) {
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = apply_op<OP>(v[2 * i], bf16_lo(x[i]));
      v[2 * i + 1] = apply_op<OP>(v[2 * i + 1], bf16_hi(x[i]));
    }
  }
  __device__ __forceinline__ u32x4 store() const {
    u32x4 r;
    for (int i = 0; i < 4; ++i) r[i] = pk_bf16(v[2 * i], v[2 * i + 1]);
    return r;
  }
};

template <> struct VecAcc<DT_F16> {
  static constexpr int N = 8;
  float v[8];
  __device__ __forceinline__ static float h2f(uint32_t bits) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)bits);
  }
  __device__ __forceinline__ static uint32_t f2h(float f) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f);
  }
  __device__ __forceinline__ void load(u32x4 x) {
    for (int i = 0; i < 4; ++i) { v[2 * i] = h2f(x[i] & 0xffff); v[2 * i + 1] = h2f(x[i] >> 16); }
  }
  template <int OP> __device__ __forceinline__ void acc(u32x4 x) {
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = apply_op<OP>(v[2 * i], h2f(x[i] & 0xffff));
      v[2 * i + 1] = apply_op<OP>(v[2 * i + 1], h2f(x[i] >> 16));
    }
  }
  __device__ __forceinline__ u32x4 store() const {
    u32x4 r;
    for (int i = 0; i < 4; ++i) r[i] = f2h(v[2 * i]) | (f2h(v[2 * i + 1]) << 16);
    return r;
  }
};

template <> struct VecAcc<DT_F64> {
  static constexpr int N = 2;
  double v[2];
  __device__ __forceinline__ static double d(uint32_t lo, uint32_t hi) {
    return __hiloint2double((int)hi, (int)lo);
  }
  __device__ __forceinline__ void load(u32x4 x) { v[0] = d(x[0], x[1]); v[1] = d(x[2], x[3]); }
  template <int OP> __device__ __forceinline__ void acc(u32x4 x) {
    v[0] = apply_op<OP>(v[0], d(x[0], x[1]));
    v[1] = apply_op<OP>(v[1], d(x[2], x[3]));
  }
  __device__ __forceinline__ u32x4 store() const {
    u32x4 r;
    r[0] = (uint32_t)__double2loint(v[0]); r[1] = (uint32_t)__double2hiint(v[0]);
    r[2] = (uint32_t)__double2loint(v[1]); r[3] = (uint32_t)__double2hiint(v[1]);
    return r;
  }
};

template <> struct VecAcc<DT_I32> {
  static constexpr int N = 4;
  int32_t v[4];
  __device__ __forceinline__ void load(u32x4 x) { for (int i = 0; i < 4; ++i) v[i] = (int32_t)x[i]; }
  template <int OP> __device__ __forceinline__ void acc(u32x4 x) {
    for (int i = 0; i < 4; ++i) v[i] = apply_op<OP>(v[i], (int32_t)x[i]);
  }
  __device__ __forceinline__ u32x4 store() const { u32x4 r; for (int i = 0; i < 4; ++i) r[i] = (uint32_t)v[i]; return r; }
};

template <> struct VecAcc<DT_I64> {
  static constexpr int N = 2;
  int64_t v[2];
  __device__ __forceinline__ static int64_t q(uint32_t lo, uint32_t hi) { return (int64_t)(((uint64_t)hi << 32) | lo); }
  __device__ __forceinline__ void load(u32x4 x) { v[0] = q(x[0], x[1]); v[1] = q(x[2], x[3]); }
  template <int OP> __device__ __forceinline__ void acc(u32x4 x) {
    v[0] = apply_op<OP>(v[0], q(x[0], x[1]));
    v[1] = apply_op<OP>(v[1], q(x[2], x[3]));
  }
  __device__ __forceinline__ u32x4 store() const {
    u32x4 r;
    r[0] = (uint32_t)v[0]; r[1] = (uint32_t)((uint64_t)v[0] >> 32);
    r[2] = (uint32_t)v[1]; r[3] = (uint32_t)((uint64_t)v[1] >> 32);
    return r;
  }
};

// Dispatch helper: calls f.template operator()<DT, OP>() for a supported pair.
template <typename F>
inline void dispatch_dt_op(int dt, int op, F&& f) {
#define CCMPI_OPS(D)                                              \
  switch (op) {                                                   \
    case OP_SUM: f.template operator()<D, OP_SUM>(); return;      \
    case OP_PROD: f.template operator()<D, OP_PROD>(); return;    \
    case OP_MIN: f.template operator()<D, OP_MIN>(); return;      \
    case OP_MAX: f.template operator()<D, OP_MAX>(); return;      \
  }                                                               \
  break;
  switch (dt) {
    case DT_F32: CCMPI_OPS(DT_F32)
    case DT_BF16: CCMPI_OPS(DT_BF16)
    case DT_F16: CCMPI_OPS(DT_F16)
    case DT_F64: CCMPI_OPS(DT_F64)
    case DT_I32: CCMPI_OPS(DT_I32)
    case DT_I64: CCMPI_OPS(DT_I64)
  }
#undef CCMPI_OPS
  throw std::invalid_argument("ccmpi device: unsupported (dtype, op) = (" + std::to_string(dt) + ", " +
                              std::to_string(op) + ")");
}

inline bool device_reduce_supported(int dt, int op) {
  bool dok = dt == DT_F32 || dt == DT_BF16 || dt == DT_F16 || dt == DT_F64 || dt == DT_I32 || dt == DT_I64;
  return dok && op >= OP_SUM && op <= OP_MAX;
}

}  // namespace dev
}  // namespace ccmpi
