// Hand-written collectives over IPC-mapped peer HBM (xGMI on an 8x MI355X node;
// same-device peers when several ranks share one GPU).
//
// Reference semantics they implement (mpi_wrapper/comm.py):
//   Allreduce      :18-22   -> allreduce_{oneshot,twoshot}; reduce_bcast = the
//                              reference's own myAllreduce algorithm (:63-107)
//   Allgather      :24-29   -> allgather (pull)
//   Reduce_scatter :31-36   -> reduce_scatter (block), pull + in-register sum
//   Alltoall       :41-61   -> alltoall (pull), also myAlltoall / myAlltoall2 (:110-199)
//   (+ bcast, used by the façade and the harness)
//
// Structure shared by every kernel (one CTA = "block" b):
//   1. publish: lane j (< nranks) writes this rank's buffer codes into rank j's
//      signal buffer at [block b][my rank], release, then the phase-0 flag = epoch.
//   2. wait until all ranks' phase-0 flags for block b reach epoch (bounded spin).
//   3. body: CTA b works on its contiguous share of the vectors, reading peers
//      with system-coherent 16-B buffer loads (every peer's bytes in flight at
//      once: all 7 xGMI links busy), reducing in registers in rank order
//      0..p-1 (deterministic, bitwise identical on every rank).
//   4. phase flags between dependent stages (two-shot) and a final flag so no
//      rank returns (and lets its buffers be overwritten) while a peer still
//      reads them.
// Block b only ever waits for block b of its peers, so there is no grid-wide
// barrier; grids are sized identically on all ranks from (bytes, nranks).
// Reductions through LDS add a round trip without reuse (each byte is read
// once), so partial sums stay in VGPRs; the LDS-DMA-staged variant
// (reduce_span_lds, algo "fanout_lds") measured even or slower on one GPU
// (profiles/r2_coll/lds_reduce.md) and is kept as a bench candidate for xGMI.
#include <cstdlib>

#include "common.hpp"
#include "collectives.hpp"

namespace ccmpi {
namespace dev {

namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 2;

struct BlockRange {
  uint64_t lo, hi;
};

__device__ __forceinline__ BlockRange split_range(uint64_t n, int parts, int idx) {
  uint64_t per = (n + parts - 1) / parts;
  uint64_t lo = per * idx;
  uint64_t hi = lo + per;
  if (lo > n) lo = n;
  if (hi > n) hi = n;
  return {lo, hi};
}


// Per-CTA prologue: bump the epoch, publish up to two buffer codes, barrier.
// Returns false on timeout.  `codes` (LDS) receives every rank's codes.
__device__ bool start_phase(const CollArgs& a, uint64_t* s_epoch, uint64_t (*codes)[kMaxRanks]) {
  const PeerTable* pt = a.pt;
  const int b = blockIdx.x, t = threadIdx.x, me = pt->rank, nr = pt->size;
  if (t == 0) *s_epoch = a.epochs[b] + 1;
  __syncthreads();
  const uint64_t e = *s_epoch;
  Signals* mine = pt->sig[me];
  if (t < nr) {
    Signals* peer = pt->sig[t];
    signal_store(&peer->addr[0][b][me], a.src_code);
    signal_store(&peer->addr[1][b][me], a.res_code);
    // make every prior write of this rank (earlier kernels' output in this
    // XCD's L2, e.g. the tensor we are about to publish) visible system-wide
    release_sys();
    signal_store(&peer->flag[0][b][me], e);
  }
  bool ok = true;
  if (t < nr) {
    ok = wait_geq(&mine->flag[0][b][t], e, a.timeout_ticks, &mine->error, 0x100 + t);
    if (!ok) report_host(pt, 0x100 + t);
    if (ok) {
      codes[0][t] = __hip_atomic_load(&mine->addr[0][b][t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      codes[1][t] = __hip_atomic_load(&mine->addr[1][b][t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  ok = __syncthreads_and(ok);
  return ok;
}

// Stage flag `phase` (1..3): every thread's stores are drained, then lane j
// tells rank j, then we wait for all ranks.  Returns false on timeout.
__device__ bool sync_phase(const CollArgs& a, int phase, uint64_t e) {
  const PeerTable* pt = a.pt;
  const int b = blockIdx.x, t = threadIdx.x, me = pt->rank, nr = pt->size;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  Signals* mine = pt->sig[me];
  if (t < nr) {
    release_sys();
    signal_store(&pt->sig[t]->flag[phase][b][me], e);
  }
  bool ok = true;
  if (t < nr) {
    ok = wait_geq(&mine->flag[phase][b][t], e, a.timeout_ticks, &mine->error, 0x100 * (phase + 1) + t);
    if (!ok) report_host(pt, 0x100 * (phase + 1) + t);
  }
  ok = __syncthreads_and(ok);
  return ok;
}

__device__ __forceinline__ void finish(const CollArgs& a, uint64_t e) {
  if (threadIdx.x == 0) a.epochs[blockIdx.x] = e;
}

// ---------------------------------------------------------------------------
// scalar element helpers for the (< 16 B) tail of reductions
// ---------------------------------------------------------------------------
template <int DT> struct Elem;
template <> struct Elem<DT_F32> { using A = float; static constexpr int B = 4;
  __device__ static A ld(Rsrc r, uint32_t o) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r.r, o, 0, kCachePolicySys)); }
  __device__ static void st(Rsrc r, uint32_t o, A v) { __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r.r, o, 0, kStorePolicy); } };
template <> struct Elem<DT_I32> { using A = int32_t; static constexpr int B = 4;
  __device__ static A ld(Rsrc r, uint32_t o) { return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r.r, o, 0, kCachePolicySys); }
  __device__ static void st(Rsrc r, uint32_t o, A v) { __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, r.r, o, 0, kStorePolicy); } };
template <> struct Elem<DT_BF16> { using A = float; static constexpr int B = 2;
  __device__ static A ld(Rsrc r, uint32_t o) { return __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r.r, o, 0, kCachePolicySys) << 16); }
  __device__ static void st(Rsrc r, uint32_t o, A v) { __builtin_amdgcn_raw_buffer_store_b16((uint16_t)f32_to_bf16_bits(v), r.r, o, 0, kStorePolicy); } };
template <> struct Elem<DT_F16> { using A = float; static constexpr int B = 2;
  __device__ static A ld(Rsrc r, uint32_t o) { return (float)__builtin_bit_cast(_Float16, (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r.r, o, 0, kCachePolicySys)); }
  __device__ static void st(Rsrc r, uint32_t o, A v) { __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (_Float16)v), r.r, o, 0, kStorePolicy); } };
template <> struct Elem<DT_F64> { using A = double; static constexpr int B = 8;
  __device__ static A ld(Rsrc r, uint32_t o) { auto v = __builtin_amdgcn_raw_buffer_load_b64(r.r, o, 0, kCachePolicySys); return __hiloint2double((int)v[1], (int)v[0]); }
  __device__ static void st(Rsrc r, uint32_t o, A v) { typedef unsigned u2 __attribute__((ext_vector_type(2))); u2 x; x[0] = (uint32_t)__double2loint(v); x[1] = (uint32_t)__double2hiint(v); __builtin_amdgcn_raw_buffer_store_b64(x, r.r, o, 0, kStorePolicy); } };
template <> struct Elem<DT_I64> { using A = int64_t; static constexpr int B = 8;
  __device__ static A ld(Rsrc r, uint32_t o) { auto v = __builtin_amdgcn_raw_buffer_load_b64(r.r, o, 0, kCachePolicySys); return (int64_t)(((uint64_t)v[1] << 32) | v[0]); }
  __device__ static void st(Rsrc r, uint32_t o, A v) { typedef unsigned u2 __attribute__((ext_vector_type(2))); u2 x; x[0] = (uint32_t)v; x[1] = (uint32_t)((uint64_t)v >> 32); __builtin_amdgcn_raw_buffer_store_b64(x, r.r, o, 0, kStorePolicy); } };

// Reduce bytes [off, off+len) of every rank's buffer (codes[j]) and store the
// result into outs[0] (FAN = false, local) or into every outs[j], j < size
// (FAN = true: local + peer-mapped outputs, the all-gather done as posted
// writes).  Vector part by all threads; element tail by thread 0.
template <int DT, int OP, int NRM, bool FAN>
__device__ void reduce_span_to(const PeerTable* pt, const uint64_t* codes, uint64_t off, uint64_t len,
                               char* const* outs) {
  const int nr = pt->size;
  const int nout = FAN ? nr : 1;
  const uint64_t vbytes = len & ~15ull;
  // process in windows of < 2 GiB so 32-bit voffsets suffice
  const uint64_t kWin = 1ull << 30;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    Rsrc src[NRM];
#pragma unroll
    for (int j = 0; j < NRM; ++j)
      if (j < nr) src[j] = make_rsrc(uniform_ptr(resolve(pt, j, codes[j]) + off + w), wl);
    Rsrc out[FAN ? NRM : 1];
#pragma unroll
    for (int j = 0; j < (FAN ? NRM : 1); ++j)
      if (j < nout) out[j] = make_rsrc(uniform_ptr(outs[j] + w), wl);
    const uint32_t nv = wl / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads * kUnroll) {
      VecAcc<DT> acc[kUnroll];
      u32x4 x[kUnroll][NRM];
#pragma unroll
      for (int j = 0; j < NRM; ++j) {
        if (j < nr) {
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) {
            uint32_t vv = v + u * kThreads;
            if (vv < nv) x[u][j] = ld16(src[j], vv * 16);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        uint32_t vv = v + u * kThreads;
        if (vv < nv) {
          acc[u].load(x[u][0]);
#pragma unroll
          for (int j = 1; j < NRM; ++j)
            if (j < nr) acc[u].template acc<OP>(x[u][j]);
          const u32x4 r = acc[u].store();
#pragma unroll
          for (int j = 0; j < (FAN ? NRM : 1); ++j)
            if (j < nout) st16(out[j], vv * 16, r);
        }
      }
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    using E = Elem<DT>;
    for (uint32_t o = 0; o < tail; o += E::B) {
      typename E::A acc = E::ld(make_rsrc(resolve(pt, 0, codes[0]) + off + vbytes, (uint32_t)tail), o);
      for (int j = 1; j < nr; ++j)
        acc = apply_op<OP>(acc, E::ld(make_rsrc(resolve(pt, j, codes[j]) + off + vbytes, (uint32_t)tail), o));
      for (int j = 0; j < nout; ++j) E::st(make_rsrc(outs[j] + vbytes, (uint32_t)tail), o, acc);
    }
  }
}

// LDS-staged variant of reduce_span_to (algo "fanout_lds"): every
// source's 16-B vectors go peer HBM -> LDS by DMA (buffer_load_dwordx4 ... lds,
// no VGPRs held while in flight), double-buffered one tile (kThreads vectors per
// source) ahead; each lane reads back only the vectors its own DMA lane wrote, so
// no barrier is needed.  LDS: 2 x NRM x 4 KiB per CTA.  Measured against the
// register path in profiles/r2_coll/lds_reduce.md.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int DT, int OP, int NRM, bool FAN>
__device__ void reduce_span_lds(const PeerTable* pt, const uint64_t* codes, uint64_t off, uint64_t len,
                                char* const* outs) {
  __shared__ __attribute__((aligned(16))) char stage[2][NRM][kThreads * 16];
  const int nr = pt->size;
  const int nout = FAN ? nr : 1;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t my = threadIdx.x * 16;
  const uint64_t vbytes = len & ~15ull;
  const uint64_t kWin = 1ull << 30;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    Rsrc src[NRM];
#pragma unroll
    for (int j = 0; j < NRM; ++j)
      if (j < nr) src[j] = make_rsrc(uniform_ptr(resolve(pt, j, codes[j]) + off + w), wl);
    Rsrc out[FAN ? NRM : 1];
#pragma unroll
    for (int j = 0; j < (FAN ? NRM : 1); ++j)
      if (j < nout) out[j] = make_rsrc(uniform_ptr(outs[j] + w), wl);
    const uint32_t nv = wl / 16, ntiles = (nv + kThreads - 1) / kThreads;
    auto issue = [&](uint32_t t, int buf) {
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr)  // out-of-range lanes read 0 (buffer bounds), never stored
          __builtin_amdgcn_raw_ptr_buffer_load_lds(src[j].r, (lds_ptr_t)&stage[buf][j][wave * 1024], 16,
                                                   t * kThreads * 16 + my, 0, 0, kCachePolicySys);
    };
    if (ntiles) issue(0, 0);
    for (uint32_t t = 0; t < ntiles; ++t) {
      const int buf = t & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u32x4 x[NRM];
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr) x[j] = *reinterpret_cast<const u32x4*>(&stage[buf][j][my]);
      if (t + 1 < ntiles) issue(t + 1, buf ^ 1);
      const uint32_t vv = t * kThreads + threadIdx.x;
      if (vv < nv) {
        VecAcc<DT> acc;
        acc.load(x[0]);
#pragma unroll
        for (int j = 1; j < NRM; ++j)
          if (j < nr) acc.template acc<OP>(x[j]);
        const u32x4 r = acc.store();
#pragma unroll
        for (int j = 0; j < (FAN ? NRM : 1); ++j)
          if (j < nout) st16(out[j], vv * 16, r);
      }
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    using E = Elem<DT>;
    for (uint32_t o = 0; o < tail; o += E::B) {
      typename E::A acc = E::ld(make_rsrc(resolve(pt, 0, codes[0]) + off + vbytes, (uint32_t)tail), o);
      for (int j = 1; j < nr; ++j)
        acc = apply_op<OP>(acc, E::ld(make_rsrc(resolve(pt, j, codes[j]) + off + vbytes, (uint32_t)tail), o));
      for (int j = 0; j < nout; ++j) E::st(make_rsrc(outs[j] + vbytes, (uint32_t)tail), o, acc);
    }
  }
}

template <int DT, int OP, int NRM>
__device__ __forceinline__ void reduce_span(const PeerTable* pt, const uint64_t* codes, uint64_t off, uint64_t len,
                                            uint64_t total_bytes, char* dst) {
  char* const outs[1] = {dst};
  reduce_span_to<DT, OP, NRM, false>(pt, codes, off, len, outs);
  (void)total_bytes;
}

// Copy bytes [0,len) from `src` (any mapped address) to `dst` (local).
__device__ void copy_span(const char* src, char* dst, uint64_t len) {
  const uint64_t kWin = 1ull << 30;
  const uint64_t vbytes = len & ~15ull;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    Rsrc s = make_rsrc(uniform_ptr(const_cast<char*>(src) + w), wl);
    Rsrc d = make_rsrc(uniform_ptr(dst + w), wl);
    const uint32_t nv = wl / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads * 4) {
      u32x4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (v + u * kThreads < nv) x[u] = ld16(s, (v + u * kThreads) * 16);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (v + u * kThreads < nv) st16(d, (v + u * kThreads) * 16, x[u]);
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    Rsrc s = make_rsrc(const_cast<char*>(src) + vbytes, (uint32_t)tail);
    Rsrc d = make_rsrc(dst + vbytes, (uint32_t)tail);
    for (uint32_t o = 0; o < tail; ++o)
      __builtin_amdgcn_raw_buffer_store_b8(__builtin_amdgcn_raw_buffer_load_b8(s.r, o, 0, kCachePolicySys), d.r, o, 0, kStorePolicy);
  }
}

// Copy from several peers at once: dst_j <- src_j for j in [0,nr) except skip.
// Keeps all peers' loads in flight together (all links busy).
template <int NRM>
__device__ void gather_spans(const char* const* srcs, char* const* dsts, int nr, int skip, uint64_t len) {
  const uint64_t kWin = 1ull << 30;
  const uint64_t vbytes = len & ~15ull;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    Rsrc s[NRM], d[NRM];
#pragma unroll
    for (int j = 0; j < NRM; ++j) {
      if (j < nr && j != skip) {
        s[j] = make_rsrc(uniform_ptr(const_cast<char*>(srcs[j]) + w), wl);
        d[j] = make_rsrc(uniform_ptr(dsts[j] + w), wl);
      }
    }
    const uint32_t nv = wl / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads * kUnroll) {
      u32x4 x[kUnroll][NRM];
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr && j != skip)
#pragma unroll
          for (int u = 0; u < kUnroll; ++u)
            if (v + u * kThreads < nv) x[u][j] = ld16(s[j], (v + u * kThreads) * 16);
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr && j != skip)
#pragma unroll
          for (int u = 0; u < kUnroll; ++u)
            if (v + u * kThreads < nv) st16(d[j], (v + u * kThreads) * 16, x[u][j]);
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    for (int j = 0; j < nr; ++j) {
      if (j == skip) continue;
      Rsrc s = make_rsrc(const_cast<char*>(srcs[j]) + vbytes, (uint32_t)tail);
      Rsrc d = make_rsrc(dsts[j] + vbytes, (uint32_t)tail);
      for (uint32_t o = 0; o < tail; ++o)
        __builtin_amdgcn_raw_buffer_store_b8(__builtin_amdgcn_raw_buffer_load_b8(s.r, o, 0, kCachePolicySys), d.r, o, 0, kStorePolicy);
    }
  }
}

// Copy one local span to several destinations (push all-gather): each 16-B
// vector is loaded once and stored to every dsts[j], j != skip.
template <int NRM>
__device__ void fanout_span(const char* src, char* const* dsts, int nr, int skip, uint64_t len) {
  constexpr int kFanUnroll = 4;  // one load feeds p stores: deeper than kUnroll
  const uint64_t kWin = 1ull << 30;
  const uint64_t vbytes = len & ~15ull;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    Rsrc s = make_rsrc(uniform_ptr(const_cast<char*>(src) + w), wl);
    Rsrc d[NRM];
#pragma unroll
    for (int j = 0; j < NRM; ++j)
      if (j < nr && j != skip) d[j] = make_rsrc(uniform_ptr(dsts[j] + w), wl);
    const uint32_t nv = wl / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads * kFanUnroll) {
      u32x4 x[kFanUnroll];
#pragma unroll
      for (int u = 0; u < kFanUnroll; ++u)
        if (v + u * kThreads < nv) x[u] = ld16(s, (v + u * kThreads) * 16);
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr && j != skip)
#pragma unroll
          for (int u = 0; u < kFanUnroll; ++u)
            if (v + u * kThreads < nv) st16(d[j], (v + u * kThreads) * 16, x[u]);
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    Rsrc s = make_rsrc(const_cast<char*>(src) + vbytes, (uint32_t)tail);
    for (int j = 0; j < nr; ++j) {
      if (j == skip) continue;
      Rsrc d = make_rsrc(dsts[j] + vbytes, (uint32_t)tail);
      for (uint32_t o = 0; o < tail; ++o)
        __builtin_amdgcn_raw_buffer_store_b8(__builtin_amdgcn_raw_buffer_load_b8(s.r, o, 0, kCachePolicySys), d.r, o, 0, kStorePolicy);
    }
  }
}

// Reduce `nr` slots at base + j*stride (this rank's memory) and store the
// result into every outs[j] (local or peer-mapped); ONE: into outs[0] only.
template <int DT, int OP, int NRM, bool ONE = false>
__device__ void reduce_fanout(const char* base, uint64_t stride, int nr, uint64_t len, char* const* outs) {
  const int nout = ONE ? 1 : nr;
  const uint64_t vbytes = len & ~15ull;
  const uint64_t kWin = 1ull << 30;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    Rsrc src[NRM], dst[NRM];
#pragma unroll
    for (int j = 0; j < NRM; ++j) {
      if (j < nr) {
        src[j] = make_rsrc(uniform_ptr(const_cast<char*>(base) + j * stride + w), wl);
        if (j < nout) dst[j] = make_rsrc(uniform_ptr(outs[j] + w), wl);
      }
    }
    const uint32_t nv = wl / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads * kUnroll) {
      u32x4 x[kUnroll][NRM];
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr)
#pragma unroll
          for (int u = 0; u < kUnroll; ++u)
            if (v + u * kThreads < nv) x[u][j] = ld16(src[j], (v + u * kThreads) * 16);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (v + u * kThreads < nv) {
          VecAcc<DT> acc;
          acc.load(x[u][0]);
#pragma unroll
          for (int j = 1; j < NRM; ++j)
            if (j < nr) acc.template acc<OP>(x[u][j]);
          const u32x4 r = acc.store();
#pragma unroll
          for (int j = 0; j < NRM; ++j)
            if (j < nout) st16(dst[j], (v + u * kThreads) * 16, r);
        }
      }
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    using E = Elem<DT>;
    for (uint32_t o = 0; o < tail; o += E::B) {
      typename E::A acc = E::ld(make_rsrc(const_cast<char*>(base) + vbytes, (uint32_t)tail), o);
      for (int j = 1; j < nr; ++j)
        acc = apply_op<OP>(acc, E::ld(make_rsrc(const_cast<char*>(base) + j * stride + vbytes, (uint32_t)tail), o));
      for (int j = 0; j < nout; ++j) E::st(make_rsrc(outs[j] + vbytes, (uint32_t)tail), o, acc);
    }
  }
}

// Element-aligned partition of `nbytes` into `parts` pieces whose boundaries
// are multiples of 16 B (except the end).
__device__ __forceinline__ BlockRange part16(uint64_t nbytes, int parts, int idx) {
  uint64_t nv = (nbytes + 15) / 16;
  BlockRange r = split_range(nv, parts, idx);
  r.lo *= 16;
  r.hi *= 16;
  if (r.hi > nbytes) r.hi = nbytes;
  if (r.lo > nbytes) r.lo = nbytes;
  return r;
}

}  // namespace

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------

// One-shot: each rank reads the whole buffer from every rank and reduces.
template <int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_allreduce_oneshot(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  BlockRange r = part16(a.nbytes, gridDim.x, blockIdx.x);
  if (r.hi > r.lo) reduce_span<DT, OP, NRM>(a.pt, codes[0], r.lo, r.hi - r.lo, a.nbytes, a.out + r.lo);
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Two-shot: reduce-scatter (rank r owns shard r) into the published result
// buffer, phase barrier, then all-gather of the shards into `out`.
template <int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_allreduce_twoshot(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  // shard boundaries (16-B aligned), then this CTA's slice of each shard
  BlockRange mys = part16(a.nbytes, nr, me);
  BlockRange sub = part16(mys.hi - mys.lo, gridDim.x, blockIdx.x);
  char* res_local = resolve(pt, me, codes[1][me]);
  if (sub.hi > sub.lo)
    reduce_span<DT, OP, NRM>(pt, codes[0], mys.lo + sub.lo, sub.hi - sub.lo, a.nbytes, res_local + mys.lo + sub.lo);
  if (!sync_phase(a, 1, e)) return;
  // all-gather: shard j's slice `blockIdx` lives in rank j's result buffer
  __shared__ const char* srcs[kMaxRanks];
  __shared__ char* dsts[kMaxRanks];
  __shared__ uint64_t lens[kMaxRanks];
  if (threadIdx.x < nr) {
    int j = threadIdx.x;
    BlockRange sj = part16(a.nbytes, nr, j);
    BlockRange bj = part16(sj.hi - sj.lo, gridDim.x, blockIdx.x);
    srcs[j] = resolve(pt, j, codes[1][j]) + sj.lo + bj.lo;
    dsts[j] = a.out + sj.lo + bj.lo;
    lens[j] = bj.hi - bj.lo;
  }
  __syncthreads();
  // shard slices differ by at most 16 B between ranks: copy the common length
  // for everybody at once, then the stragglers individually.
  uint64_t common = lens[0];
  for (int j = 1; j < nr; ++j) common = min(common, lens[j]);
  const int skip = (a.out == res_local) ? me : -1;
  if (common) gather_spans<NRM>(srcs, dsts, nr, skip, common);
  for (int j = 0; j < nr; ++j)
    if (j != skip && lens[j] > common) copy_span(srcs[j] + common, dsts[j] + common, lens[j] - common);
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}


// Fan-out two-shot: one phase.  Rank r pulls shard r's slice from every rank
// (reads, rank order), reduces it and stores the result straight into EVERY
// rank's result buffer (codes[1][j], local + posted peer writes): the
// all-gather rides on the reduce-scatter's stores, so there is no middle
// barrier and no second read of the shards.  HBM traffic per rank: S read +
// S written (pull two-shot: S read + S/p written, then S read + S written
// again for the all-gather).  In place is safe: only rank r reads or writes
// region r of any buffer, and each CTA reads its slice before it writes it.
template <int DT, int OP, int NRM, bool LDS = false>
__global__ void __launch_bounds__(kThreads) k_allreduce_twoshot_fanout(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  BlockRange mys = part16(a.nbytes, nr, me);
  BlockRange sub = part16(mys.hi - mys.lo, gridDim.x, blockIdx.x);
  if (sub.hi > sub.lo) {
    __shared__ char* outs[kMaxRanks];
    if (threadIdx.x < nr) outs[threadIdx.x] = resolve(pt, threadIdx.x, codes[1][threadIdx.x]) + mys.lo + sub.lo;
    __syncthreads();
    if constexpr (LDS)
      reduce_span_lds<DT, OP, NRM, true>(pt, codes[0], mys.lo + sub.lo, sub.hi - sub.lo, outs);
    else
      reduce_span_to<DT, OP, NRM, true>(pt, codes[0], mys.lo + sub.lo, sub.hi - sub.lo, outs);
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Push two-shot: phase 1 writes my slice of shard j into rank j's inbox slot
// [me] (remote 16-B sc0|sc1 stores: posted writes, no round trip); after the
// phase flag, rank j reduces its p inbox slots (local reads, rank order) and
// writes the reduced slice into EVERY rank's output (the all-gather is pushed
// too).  Same bytes on the wire as the pull form; which one a fabric prefers
// is measured at run time (bench/autotune candidates).
template <int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_allreduce_twoshot_push(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  const char* src = a.in;  // local input; codes[0][j] = rank j's inbox, codes[1][j] = its result
  const uint64_t shard = (((a.nbytes + nr - 1) / nr) + 15) / 16 * 16;  // inbox slot stride
  // ---- phase 1: scatter my input shards into the owners' inboxes
  {
    __shared__ char* dsts[kMaxRanks];
    __shared__ const char* srcs[kMaxRanks];
    __shared__ uint64_t lens[kMaxRanks];
    if (threadIdx.x < nr) {
      const int j = threadIdx.x;
      BlockRange sj = part16(a.nbytes, nr, j);
      BlockRange bj = part16(sj.hi - sj.lo, gridDim.x, blockIdx.x);
      srcs[j] = src + sj.lo + bj.lo;
      dsts[j] = resolve(pt, j, codes[0][j]) + (uint64_t)me * shard + bj.lo;
      lens[j] = bj.hi - bj.lo;
    }
    __syncthreads();
    uint64_t common = lens[0];
    for (int j = 1; j < nr; ++j) common = min(common, lens[j]);
    if (common) gather_spans<NRM>(srcs, dsts, nr, -1, common);
    for (int j = 0; j < nr; ++j)
      if (lens[j] > common) copy_span(srcs[j] + common, dsts[j] + common, lens[j] - common);
  }
  if (!sync_phase(a, 1, e)) return;
  // ---- phase 2: reduce my inbox slots (rank order), store the result slice into
  //      every rank's output directly (local + 7 remote posted writes)
  BlockRange mys = part16(a.nbytes, nr, me);
  BlockRange sub = part16(mys.hi - mys.lo, gridDim.x, blockIdx.x);
  if (sub.hi > sub.lo) {
    __shared__ char* outs[kMaxRanks];
    if (threadIdx.x < nr) outs[threadIdx.x] = resolve(pt, threadIdx.x, codes[1][threadIdx.x]) + mys.lo + sub.lo;
    __syncthreads();
    reduce_fanout<DT, OP, NRM>(resolve(pt, me, codes[0][me]) + sub.lo, shard, nr, sub.hi - sub.lo, outs);
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Inbox-to-local two-shot, the collective half of the push row-parallel GEMM
// (DeviceComm::gemm_push_rowpar): every rank's GEMM epilogue has already stored its
// partial of shard j (row block j) into rank j's inbox slot [rank] as posted writes,
// so the reduce-scatter's traffic crossed the fabric under the GEMM.  Here rank r
// reduces its p slots (local reads, rank order) into its own slot r, and after the
// phase flag every rank pulls every reduced shard from its owner into `out`
// (a local tensor).  codes[0][j] = rank j's inbox; slot stride = the shard size.
template <int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_allreduce_inbox_local(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  const uint64_t shard = (((a.nbytes + nr - 1) / nr) + 15) / 16 * 16;
  {
    BlockRange mys = part16(a.nbytes, nr, me);
    BlockRange sub = part16(mys.hi - mys.lo, gridDim.x, blockIdx.x);
    char* inbox = resolve(pt, me, codes[0][me]);
    if (sub.hi > sub.lo) {
      char* outs[1] = {inbox + (uint64_t)me * shard + sub.lo};
      reduce_fanout<DT, OP, NRM, true>(inbox + sub.lo, shard, nr, sub.hi - sub.lo, outs);
    }
  }
  if (!sync_phase(a, 1, e)) return;
  __shared__ const char* srcs[kMaxRanks];
  __shared__ char* dsts[kMaxRanks];
  __shared__ uint64_t lens[kMaxRanks];
  if (threadIdx.x < nr) {
    const int j = threadIdx.x;
    BlockRange sj = part16(a.nbytes, nr, j);
    BlockRange bj = part16(sj.hi - sj.lo, gridDim.x, blockIdx.x);
    srcs[j] = resolve(pt, j, codes[0][j]) + (uint64_t)j * shard + bj.lo;
    dsts[j] = a.out + sj.lo + bj.lo;
    lens[j] = bj.hi - bj.lo;
  }
  __syncthreads();
  uint64_t common = lens[0];
  for (int j = 1; j < nr; ++j) common = min(common, lens[j]);
  if (common) gather_spans<NRM>(srcs, dsts, nr, -1, common);
  for (int j = 0; j < nr; ++j)
    if (lens[j] > common) copy_span(srcs[j] + common, dsts[j] + common, lens[j] - common);
  // no rank's next push may land in an inbox a peer still reads
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Inbox-to-mean: the TP sum of the per-token fc_o output z followed by the mean over each
// sequence's S rows (the harness logits), as reduce-scatter + mean + all-gather of the means.
// Every rank's attention kernel has pushed its partial z row block j into rank j's inbox slot
// [rank] (posted writes under the attention); here rank r sums its p slots per row (rank
// order), averages each sequence's S rows (row order), and stores the B / p mean rows into
// EVERY rank's logits buffer (local + peer-mapped write-through stores).  So the fabric
// carries (p-1)/p of z once plus B x 16 logits -- not z twice (all-reduce) -- and the
// separate mean kernel disappears.  a.nbytes = the whole z (B*S x 16 fp32), a.root = S,
// codes[0][j] = rank j's inbox (slot stride nbytes / p), codes[1][j] = rank j's logits
// (B x 16 fp32, symmetric).
template <int NRM>
__global__ void __launch_bounds__(kThreads) k_inbox_mean(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size, S = a.root;
  const uint32_t shard = (uint32_t)(a.nbytes / nr), ngroups = shard / (uint32_t)(S * 64);
  {
    char* inbox = resolve(pt, me, codes[0][me]);
    Rsrc src[NRM], dst[NRM];
#pragma unroll
    for (int j = 0; j < NRM; ++j)
      if (j < nr) {
        src[j] = make_rsrc(uniform_ptr(inbox + (uint64_t)j * shard), shard);
        dst[j] = make_rsrc(uniform_ptr(resolve(pt, j, codes[1][j]) + (uint64_t)me * ngroups * 64), ngroups * 64);
      }
    const float n = (float)S;
    for (uint32_t idx = blockIdx.x * kThreads + threadIdx.x; idx < ngroups * 4; idx += gridDim.x * kThreads) {
      const uint32_t gl = idx >> 2, q = idx & 3;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int i = 0; i < S; ++i) {
        const uint32_t off = (gl * S + i) * 64 + q * 16;
        float row[4];
        const u32x4 x0 = ld16(src[0], off);
#pragma unroll
        for (int k = 0; k < 4; ++k) row[k] = __uint_as_float(x0[k]);
#pragma unroll
        for (int j = 1; j < NRM; ++j)
          if (j < nr) {
            const u32x4 xj = ld16(src[j], off);
#pragma unroll
            for (int k = 0; k < 4; ++k) row[k] += __uint_as_float(xj[k]);
          }
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += row[k];
      }
      const u32x4 m = {__float_as_uint(acc[0] / n), __float_as_uint(acc[1] / n), __float_as_uint(acc[2] / n),
                       __float_as_uint(acc[3] / n)};
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr) st16(dst[j], gl * 64 + q * 16, m);
    }
  }
  // every rank's means have landed everywhere, and no rank's next push can reach an inbox
  // that is still being read
  if (!sync_phase(a, 1, e)) return;
  finish(a, e);
}

// Reference algorithm (mpi_wrapper/comm.py:63-107): the root reduces every
// rank's buffer in rank order, then every other rank copies the root's result.
template <int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_allreduce_reduce_bcast(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, root = a.root;
  BlockRange r = part16(a.nbytes, gridDim.x, blockIdx.x);
  if (me == root && r.hi > r.lo)
    reduce_span<DT, OP, NRM>(pt, codes[0], r.lo, r.hi - r.lo, a.nbytes, resolve(pt, me, codes[1][me]) + r.lo);
  if (!sync_phase(a, 1, e)) return;
  if (r.hi > r.lo) {
    char* src = resolve(pt, root, codes[1][root]) + r.lo;
    if (src != a.out + r.lo) copy_span(src, a.out + r.lo, r.hi - r.lo);
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Reduce-scatter (block): out = sum_j in_j[me*nbytes : (me+1)*nbytes].
template <int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_reduce_scatter(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  BlockRange r = part16(a.nbytes, gridDim.x, blockIdx.x);
  if (r.hi > r.lo)
    reduce_span<DT, OP, NRM>(pt, codes[0], (uint64_t)pt->rank * a.nbytes + r.lo, r.hi - r.lo, a.nbytes, a.out + r.lo);
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Per-peer block moves; `nbytes` = bytes per peer block, block strides
// src_stride / dst_stride (0 = nbytes) so staged chunks of a larger tensor
// land in place without an unpack pass.
//   MODE 0 all-gather      (pull): out[j*ds] = in_j
//   MODE 1 all-to-all      (pull): out[j*ds] = in_j[me*ss]
//   MODE 2 broadcast       (pull): out = in_root
//   MODE 3 all-to-all      (push): out_j[me*ds] = in[j*ss]   (reference myAlltoall,
//          mpi_wrapper/comm.py:130-155: each segment goes straight into its
//          destination; the input never leaves this rank's memory except as
//          posted peer writes, so it needs no registration)
//   MODE 4 all-gather      (push): out_j[me*ds] = in          (same, one source block;
//          in place -- in == out[me*ds] -- skips the self copy)
//   MODE 5 broadcast       (push): out_j = in on the root, which loads each vector
//          once and stores it to the p-1 peers; the other ranks only publish
//          their buffer and wait at the end barrier
template <int MODE, int NRM>
__global__ void __launch_bounds__(kThreads) k_move(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  const uint64_t ss = a.src_stride ? a.src_stride : a.nbytes;
  const uint64_t ds = a.dst_stride ? a.dst_stride : a.nbytes;
  if ((MODE == 0 || MODE == 1 || MODE == 3) && (a.flags & 1)) {
    // peer-major: CTA b streams one peer's block (j = b % p, slice b / p of
    // gridDim / p), one source and one destination stream per CTA
    const int j = blockIdx.x % nr;
    BlockRange q = part16(a.nbytes, gridDim.x / nr, blockIdx.x / nr);
    if (q.hi > q.lo) {
      const char* src;
      char* dst;
      if (MODE == 3 || MODE == 4) {
        src = a.in + (MODE == 3 ? (uint64_t)j * ss : 0) + q.lo;
        dst = resolve(pt, j, codes[1][j]) + (uint64_t)me * ds + q.lo;
      } else {
        src = resolve(pt, j, codes[0][j]) + (MODE == 1 ? (uint64_t)me * ss : 0) + q.lo;
        dst = a.out + (uint64_t)j * ds + q.lo;
      }
      if (src != dst) copy_span(src, dst, q.hi - q.lo);
    }
    if (!sync_phase(a, 3, e)) return;
    finish(a, e);
    return;
  }
  BlockRange r = part16(a.nbytes, gridDim.x, blockIdx.x);
  if (r.hi > r.lo) {
    if (MODE == 2) {
      if (me != a.root) copy_span(resolve(pt, a.root, codes[0][a.root]) + r.lo, a.out + r.lo, r.hi - r.lo);
    } else if (MODE == 5) {
      if (me == a.root) {
        __shared__ char* bdst[kMaxRanks];
        if (threadIdx.x < nr) bdst[threadIdx.x] = resolve(pt, threadIdx.x, codes[1][threadIdx.x]) + r.lo;
        __syncthreads();
        fanout_span<NRM>(a.in + r.lo, bdst, nr, me, r.hi - r.lo);
      }
    } else {
      __shared__ const char* srcs[kMaxRanks];
      __shared__ char* dsts[kMaxRanks];
      if (threadIdx.x < nr) {
        const int j = threadIdx.x;
        if (MODE == 3 || MODE == 4) {
          srcs[j] = a.in + (MODE == 3 ? (uint64_t)j * ss : 0) + r.lo;
          dsts[j] = resolve(pt, j, codes[1][j]) + (uint64_t)me * ds + r.lo;
        } else {
          srcs[j] = resolve(pt, j, codes[0][j]) + (MODE == 1 ? (uint64_t)me * ss : 0) + r.lo;
          dsts[j] = a.out + (uint64_t)j * ds + r.lo;
        }
      }
      __syncthreads();
      if (MODE == 4)
        fanout_span<NRM>(srcs[0], dsts, nr, srcs[me] == dsts[me] ? me : -1, r.hi - r.lo);
      else
        gather_spans<NRM>(srcs, dsts, nr, -1, r.hi - r.lo);
    }
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// All-to-all with per-peer sizes (MoE token dispatch): CTA b takes a 16-B slice
// of the concatenated send buffer and writes the part of every peer segment it
// covers straight into that peer's output (posted xGMI writes, the input never
// leaves local memory) -- MODE 3's push generalised to ragged segments.  The
// grid is the same on every rank (the per-CTA flags pair CTA b with CTA b), so
// ranks with less to send run idle CTAs through the two barriers.
__global__ void __launch_bounds__(kThreads) k_alltoallv_push(VArgs v) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  const CollArgs& a = v.a;
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int nr = pt->size;
  const BlockRange r = part16(a.nbytes, gridDim.x, blockIdx.x);
  for (int j = 0; j < nr; ++j) {
    const uint64_t lo = max(r.lo, v.soff[j]), hi = min(r.hi, v.soff[j] + v.len[j]);
    if (hi > lo) copy_span(a.in + lo, resolve(pt, j, codes[1][j]) + v.doff[j] + (lo - v.soff[j]), hi - lo);
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// The same with the count matrix read on the device: after the start barrier
// every CTA loads every rank's staged count row (p + 1 int64: counts, output
// capacity) from the peers' scratch segments into LDS, derives the packed
// offsets, and pushes its slice.  A segment that is not a 16-B multiple, or that
// would overrun the receiver's capacity, is not written: the kernel records a
// fault code (0x900 + peer) that DeviceGroup.check() raises.  The grid is fixed
// by the caller (sizes are unknown on the host).
__global__ void __launch_bounds__(kThreads) k_alltoallv_dev(VDevArgs v) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  __shared__ int64_t C[kMaxRanks][kMaxRanks + 1];
  const CollArgs& a = v.a;
  if (threadIdx.x == 0) {  // published with the start barrier (thread 0 releases before its flag)
    int64_t* mine = reinterpret_cast<int64_t*>(resolve(a.pt, a.pt->rank, a.src_code));
    __hip_atomic_store(mine + a.pt->size, v.cap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  for (int t = threadIdx.x; t < nr * (nr + 1); t += kThreads) {
    const int i = t / (nr + 1), j = t % (nr + 1);
    const int64_t* row = reinterpret_cast<const int64_t*>(resolve(pt, i, codes[0][i]));
    C[i][j] = __hip_atomic_load(row + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < nr) v.recv_counts[threadIdx.x] = C[threadIdx.x][me];
  const uint64_t es = v.es;
  uint64_t total = 0;
  for (int j = 0; j < nr; ++j) total += (uint64_t)max(C[me][j], (int64_t)0) * es;
  const BlockRange r = part16(total, gridDim.x, blockIdx.x);
  uint64_t soff = 0;
  for (int j = 0; j < nr; ++j) {
    uint64_t doff = 0;
    for (int i = 0; i < me; ++i) doff += (uint64_t)max(C[i][j], (int64_t)0) * es;
    const uint64_t len = (uint64_t)max(C[me][j], (int64_t)0) * es;
    const bool ok = C[me][j] >= 0 && (soff | doff | len) % 16 == 0 && doff + len <= (uint64_t)C[j][nr] * es;
    if (!ok) {
      if (threadIdx.x == 0 && blockIdx.x == 0) {
        __hip_atomic_store(&pt->sig[me]->error, 0x900u + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        report_host(pt, 0x900u + j);
      }
    } else {
      const uint64_t lo = max(r.lo, soff), hi = min(r.hi, soff + len);
      if (hi > lo) copy_span(a.in + lo, resolve(pt, j, codes[1][j]) + doff + (lo - soff), hi - lo);
    }
    soff += len;
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// ---------------------------------------------------------------------------
// low-latency one-shot all-reduce (small messages)
// ---------------------------------------------------------------------------
// The flag travels with the data: every 4-byte payload word is pushed to every
// peer as one naturally aligned 8-byte store (word, flag), single-copy atomic,
// into the peer's LL buffer region [parity][my rank].  Each rank then polls its
// own buffer until every unit of every source carries this call's flag and
// reduces in rank order.  No start or end barrier: one write latency instead of
// three flag round trips.  Buffer reuse is safe with two parities: a rank writes
// call k+2's data into the parity it read in call k only after every peer has
// pushed call k+1's data, i.e. finished reading call k.  The call epoch is one
// device word shared by all CTAs (the last CTA to finish advances it), so the
// parity does not depend on the grid and the kernel stays graph-capturable.
// The LL buffers are uncached device memory (hipDeviceMallocUncached, like the
// signal buffers): in coarse-grained memory a peer's 8-byte stores became
// visible to the poller only after ~20 us per source (measured, 43 us for a
// 4 KiB all-reduce at 2 ranks), with uncached memory after one write latency.
template <int DT, int OP>
__global__ void __launch_bounds__(kThreads) k_allreduce_ll(CollArgs a) {
  const PeerTable* pt = a.pt;
  const int me = pt->rank, p = pt->size;
  __shared__ uint32_t s_e;
  if (threadIdx.x == 0) s_e = __hip_atomic_load(&a.ll_state[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t E = s_e, flag = E + 1;
  const uint64_t par = E & 1;
  const uint64_t nvec = a.nbytes / 16;
  const bool stamp = a.dbg && blockIdx.x == 0 && threadIdx.x == 0;
  if (stamp) a.dbg[0] = now_ticks();
  const BlockRange r = split_range(nvec, gridDim.x, blockIdx.x);
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  // push: 16 B of payload = four (word, flag) units = 32 B per peer
  // descriptors from wave-uniform bases, per-lane byte offsets (a per-lane base
  // would make the compiler waterfall every buffer instruction over the 64 lanes)
  for (uint64_t v = r.lo + threadIdx.x; v < r.hi; v += kThreads) {
    const u32x4 x = *reinterpret_cast<const u32x4*>(a.in + v * 16);
    for (int j = 0; j < p; ++j) {
      const Rsrc rd = make_rsrc(uniform_ptr(pt->ll[j] + (par * p + me) * a.ll_slot), (uint32_t)a.ll_slot);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u2 w;
        w[0] = x[i];
        w[1] = flag;
        __builtin_amdgcn_raw_buffer_store_b64(w, rd.r, (uint32_t)(v * 32 + 8 * i), 0, kStorePolicy);
      }
    }
  }
  if (stamp) a.dbg[1] = now_ticks();
  // poll + reduce (rank order): my LL buffer holds every source's units
  const char* mine = pt->ll[me];
  bool ok = true;
  for (uint64_t v = r.lo + threadIdx.x; v < r.hi && ok; v += kThreads) {
    VecAcc<DT> acc;
    for (int j = 0; j < p && ok; ++j) {
      const Rsrc rs = make_rsrc(uniform_ptr(const_cast<char*>(mine) + (par * p + j) * a.ll_slot), (uint32_t)a.ll_slot);
      u32x4 x;
      uint64_t t0 = 0;
      uint32_t spins = 0;
      for (;;) {
        bool ready = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u2 w = __builtin_amdgcn_raw_buffer_load_b64(rs.r, (uint32_t)(v * 32 + 8 * i), 0, kCachePolicySys);
          x[i] = w[0];
          ready = ready && (w[1] == flag);
        }
        if (ready) break;
        if ((++spins & 63) == 0) {
          const uint64_t t = now_ticks();
          if (t0 == 0) t0 = t;
          else if (t - t0 > a.timeout_ticks) {
            __hip_atomic_store(&pt->sig[me]->error, 0x900u + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            report_host(pt, 0x900 + j);
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (j == 0) acc.load(x);
      else acc.template acc<OP>(x);
      if (stamp && j < 14) a.dbg[2 + j] = now_ticks();
    }
    if (ok) *reinterpret_cast<u32x4*>(a.out + v * 16) = acc.store();
  }
  // the last CTA out advances the call epoch (visible to the next kernel on the stream)
  if (stamp) a.dbg[16] = now_ticks();
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(&a.ll_state[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(&a.ll_state[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.ll_state[0], E + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// pipelined schedules: ring and recursive halving/doubling
// ---------------------------------------------------------------------------
// Both push: every byte that crosses to a peer is a posted remote store into
// the peer's inbox (reduce-scatter) or its result buffer (all-gather); every
// load is local.  The buffer is cut into p chunks (part16) and every chunk
// into gridDim.x sub-slices; CTA b owns sub-slice b of every chunk, so CTA b
// of a rank only ever waits for CTA b of its ring/partner neighbours (one
// monotonic step word per (block, source): epoch * kStepsPerEpoch + step).
// Only the start barrier is all-to-all: it guarantees every peer has reached
// this collective (its previous use of the inbox / result buffer is done)
// before anybody writes into it.  No end barrier is needed: a rank finishes
// only after the last write addressed to it has been flagged, and nobody
// reads another rank's memory.

// o1 (and o2 if TWO) = RED ? op(x, y) : x over [0, len); x, y 16-B aligned.
template <int DT, int OP, bool RED, bool TWO>
__device__ void combine_span(const char* x, const char* y, char* o1, char* o2, uint64_t len) {
  constexpr int U = 4;
  const uint64_t kWin = 1ull << 30;
  const uint64_t vbytes = len & ~15ull;
  for (uint64_t w = 0; w < vbytes; w += kWin) {
    const uint32_t wl = (uint32_t)min(kWin, vbytes - w);
    const Rsrc rx = make_rsrc(uniform_ptr(const_cast<char*>(x) + w), wl);
    const Rsrc ry = make_rsrc(uniform_ptr(const_cast<char*>(RED ? y : x) + w), wl);
    const Rsrc r1 = make_rsrc(uniform_ptr(o1 + w), wl);
    const Rsrc r2 = make_rsrc(uniform_ptr((TWO ? o2 : o1) + w), wl);
    const uint32_t nv = wl / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads * U) {
      u32x4 xa[U], ya[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t vv = v + u * kThreads;
        if (vv < nv) {
          xa[u] = ld16(rx, vv * 16);
          if (RED) ya[u] = ld16(ry, vv * 16);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t vv = v + u * kThreads;
        if (vv < nv) {
          u32x4 res = xa[u];
          if (RED) {
            VecAcc<DT> acc;
            acc.load(xa[u]);
            acc.template acc<OP>(ya[u]);
            res = acc.store();
          }
          st16(r1, vv * 16, res);
          if (TWO) st16(r2, vv * 16, res);
        }
      }
    }
  }
  const uint64_t tail = len - vbytes;
  if (tail && threadIdx.x == 0) {
    const Rsrc rx = make_rsrc(const_cast<char*>(x) + vbytes, (uint32_t)tail);
    const Rsrc r1 = make_rsrc(o1 + vbytes, (uint32_t)tail);
    const Rsrc r2 = make_rsrc((TWO ? o2 : o1) + vbytes, (uint32_t)tail);
    if constexpr (RED) {
      using E = Elem<DT>;
      const Rsrc ry = make_rsrc(const_cast<char*>(y) + vbytes, (uint32_t)tail);
      for (uint32_t o = 0; o < tail; o += E::B) {
        const typename E::A v = apply_op<OP>(E::ld(rx, o), E::ld(ry, o));
        E::st(r1, o, v);
        if (TWO) E::st(r2, o, v);
      }
    } else {
      for (uint32_t o = 0; o < tail; ++o) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b8(rx.r, o, 0, kCachePolicySys);
        __builtin_amdgcn_raw_buffer_store_b8(v, r1.r, o, 0, kStorePolicy);
        if (TWO) __builtin_amdgcn_raw_buffer_store_b8(v, r2.r, o, 0, kStorePolicy);
      }
    }
  }
}

// Drain this CTA's stores, then one lane publishes `v` (release, system scope).
__device__ __forceinline__ void post_step(uint64_t* flag, uint64_t v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    release_sys();
    signal_store(flag, v);
  }
}

// One lane waits for *flag >= v (bounded); the CTA follows.  False on timeout.
__device__ __forceinline__ bool await_step(const CollArgs& a, const uint64_t* flag, uint64_t v, int peer) {
  bool ok = true;
  if (threadIdx.x == 0) {
    const PeerTable* pt = a.pt;
    ok = wait_geq(flag, v, a.timeout_ticks, &pt->sig[pt->rank]->error, 0x800 + peer);
    if (!ok) report_host(pt, 0x800 + peer);
  }
  return __syncthreads_and(ok);
}

// CTA b's sub-slice of chunk c: absolute byte range, and its offset inside the
// chunk (= inside an inbox slot).  The split is of the SLOT size, not of the
// chunk's own length: chunks differ by up to 16 B, and two rings can deliver
// different chunks into the same slot of one inbox, so the sub-slot of CTA b
// must not depend on which chunk it carries.
struct SubSlice {
  uint64_t lo, len, rel;
};
__device__ __forceinline__ SubSlice sub_slice(uint64_t nbytes, int p, int c, uint64_t slot) {
  const BlockRange ch = part16(nbytes, p, c);
  const BlockRange r = part16(slot, gridDim.x, blockIdx.x);
  const uint64_t len = ch.hi - ch.lo;
  const uint64_t lo = min(r.lo, len), hi = min(r.hi, len);
  return {ch.lo + lo, hi - lo, lo};
}

// Ring all-reduce (reduce-scatter then all-gather, 2(p-1) pipelined steps).
// CTA b runs ring k = b % nrings (i -> i + stride_k); rings with coprime
// strides use different xGMI links, so k rings drive k links per direction.
// Ring position q of this rank: chunk (q - t) is forwarded at RS step t;
// after p-1 steps the rank owns the fully reduced chunk q + 1, writes it to
// its result and its right neighbour's result, and the all-gather forwards
// what arrives.  Inbox slot t holds the partial sum received at RS step t.
template <int DT, int OP>
__global__ void __launch_bounds__(kThreads) k_allreduce_ring(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, p = pt->size, b = blockIdx.x;
  const int k = b % a.nrings;
  const int stride = a.ring_stride[k];
  const int right = (me + stride) % p, left = (me + p - stride) % p;
  const int q = (me * a.ring_inv[k]) % p;
  const uint64_t slot = a.inbox_slot, base = e * kStepsPerEpoch;
  char* out = a.out;
  char* r_out = resolve(pt, right, codes[1][right]);
  const char* inbox = resolve(pt, me, codes[0][me]);  // inboxes are published in slot 0
  char* r_inbox = resolve(pt, right, codes[0][right]);
  const uint64_t* my_flag = &pt->sig[me]->step[b][left];
  uint64_t* r_flag = &pt->sig[right]->step[b][me];
  // reduce-scatter
  for (int t = 0; t < p - 1; ++t) {
    const SubSlice s = sub_slice(a.nbytes, p, (q - t + p) % p, slot);
    if (t == 0) {
      combine_span<DT, OP, false, false>(a.in + s.lo, nullptr, r_inbox + s.rel, nullptr, s.len);
    } else {
      if (!await_step(a, my_flag, base + t, left)) return;
      combine_span<DT, OP, true, false>(a.in + s.lo, inbox + (t - 1) * slot + s.rel, r_inbox + t * slot + s.rel,
                                        nullptr, s.len);
    }
    post_step(r_flag, base + t + 1);
  }
  // last reduction: the owned chunk, written locally and into the right neighbour's result
  {
    const SubSlice s = sub_slice(a.nbytes, p, (q + 1) % p, slot);
    if (!await_step(a, my_flag, base + p - 1, left)) return;
    combine_span<DT, OP, true, true>(a.in + s.lo, inbox + (p - 2) * slot + s.rel, out + s.lo, r_out + s.lo, s.len);
    post_step(r_flag, base + p);
  }
  // all-gather: forward the chunk that arrived in the previous step
  for (int t = 1; t < p - 1; ++t) {
    const SubSlice s = sub_slice(a.nbytes, p, (q - t + 1 + p) % p, slot);
    if (!await_step(a, my_flag, base + p - 1 + t, left)) return;
    combine_span<DT, OP, false, false>(out + s.lo, nullptr, r_out + s.lo, nullptr, s.len);
    post_step(r_flag, base + p + t);
  }
  if (!await_step(a, my_flag, base + 2 * p - 2, left)) return;
  finish(a, e);
}

// Recursive halving (reduce-scatter) + recursive doubling (all-gather), p = 2^k.
// Halving step with mask m: partner = me ^ m; the current range of m*2 chunks
// splits, the half the partner keeps is pushed into its inbox (slot region of
// this step), the own half is reduced from the partner's push.  Rank r ends
// owning chunk r; the doubling steps push the owned range into the partner's
// result buffer.  log2(p) + log2(p) steps, every step on one link.
template <int DT, int OP>
__global__ void __launch_bounds__(kThreads) k_allreduce_rhd(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, p = pt->size, b = blockIdx.x;
  const uint64_t slot = a.inbox_slot, base = e * kStepsPerEpoch;
  char* out = a.out;
  const char* inbox = resolve(pt, me, codes[0][me]);  // inboxes are published in slot 0
  Signals* mine = pt->sig[me];
  int step = 0, L = 0;
  uint64_t slot_off = 0;
  for (int m = p >> 1; m >= 1; m >>= 1, ++step) {
    const int partner = me ^ m;
    const int keep = (me & m) ? L + m : L, give = (me & m) ? L : L + m;
    const char* from = step == 0 ? a.in : out;
    char* p_inbox = resolve(pt, partner, codes[0][partner]) + slot_off;
    for (int i = 0; i < m; ++i) {
      const SubSlice s = sub_slice(a.nbytes, p, give + i, slot);
      combine_span<DT, OP, false, false>(from + s.lo, nullptr, p_inbox + i * slot + s.rel, nullptr, s.len);
    }
    post_step(&pt->sig[partner]->step[b][me], base + step + 1);
    if (!await_step(a, &mine->step[b][partner], base + step + 1, partner)) return;
    for (int i = 0; i < m; ++i) {
      const SubSlice s = sub_slice(a.nbytes, p, keep + i, slot);
      combine_span<DT, OP, true, false>(from + s.lo, inbox + slot_off + i * slot + s.rel, out + s.lo, nullptr, s.len);
    }
    L = keep;
    slot_off += (uint64_t)m * slot;
  }
  for (int m = 1; m < p; m <<= 1, ++step) {
    const int partner = me ^ m;
    const int own = me & ~(m - 1);
    char* p_out = resolve(pt, partner, codes[1][partner]);
    for (int i = 0; i < m; ++i) {
      const SubSlice s = sub_slice(a.nbytes, p, own + i, slot);
      combine_span<DT, OP, false, false>(out + s.lo, nullptr, p_out + s.lo, nullptr, s.len);
    }
    post_step(&pt->sig[partner]->step[b][me], base + step + 1);
    if (!await_step(a, &mine->step[b][partner], base + step + 1, partner)) return;
  }
  finish(a, e);
}


// Pairwise all-to-all (reference myAlltoall2, mpi_wrapper/comm.py:162-199): p - 1
// rounds after the local block; in round k rank r pushes its block for
// to = r + k into to's output (posted peer writes, one peer in flight per round),
// flags it, and waits for the block from r - k before the next round -- the
// reference's Sendrecv pairing, exchange by exchange.  Every CTA moves its
// 16-B slice of each block and pairs its flags with CTA b of the peers (one
// monotonic step word per (block, source), like the ring).  The start barrier
// guarantees every peer has entered the call before anything lands in its
// output; no end barrier: a rank returns once every block addressed to it is
// flagged, and it never reads peer memory.
__global__ void __launch_bounds__(kThreads) k_alltoall_pairwise(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, p = pt->size, b = blockIdx.x;
  const uint64_t ss = a.src_stride ? a.src_stride : a.nbytes;
  const uint64_t ds = a.dst_stride ? a.dst_stride : a.nbytes;
  const uint64_t base = e * kStepsPerEpoch;
  const BlockRange q = part16(a.nbytes, gridDim.x, b);
  const uint64_t len = q.hi - q.lo;
  if (len) copy_span(a.in + (uint64_t)me * ss + q.lo, resolve(pt, me, codes[1][me]) + (uint64_t)me * ds + q.lo, len);
  for (int k = 1; k < p; ++k) {
    const int to = (me + k) % p, from = (me + p - k) % p;
    if (len) copy_span(a.in + (uint64_t)to * ss + q.lo, resolve(pt, to, codes[1][to]) + (uint64_t)me * ds + q.lo, len);
    post_step(&pt->sig[to]->step[b][me], base + k);
    if (!await_step(a, &pt->sig[me]->step[b][from], base + k, from)) return;
  }
  finish(a, e);
}

// Last-axis collectives for tensor parallelism (fused layout transform):
//   MODE 0 all-gather : out[m][j*k + c] = in_j[m][c]                (M x k shards -> M x p*k)
//   MODE 1 reduce-scat: out[m][c] = sum_j in_j[m][me*k + c]          (M x p*k      -> M x k)
// The (row, 16-B vector) index space is flattened so short rows still keep
// every lane busy; every peer's vector is loaded before any is used.
// Requires k * elem_size % 16 == 0 (checked on the host).
template <int MODE, int DT, int OP, int NRM>
__global__ void __launch_bounds__(kThreads) k_lastaxis(CollArgs a) {
  __shared__ uint64_t s_epoch;
  __shared__ uint64_t codes[2][kMaxRanks];
  if (!start_phase(a, &s_epoch, codes)) return;
  const uint64_t e = s_epoch;
  const PeerTable* pt = a.pt;
  const int me = pt->rank, nr = pt->size;
  const uint64_t rowv = a.nbytes / 16;        // vectors per k-row (nbytes = k * elem)
  const uint64_t rows = (uint64_t)a.root;     // M (passed in `root`)
  const uint64_t total = rows * rowv;
  BlockRange r = split_range(total, gridDim.x, blockIdx.x);
  __shared__ const char* base[kMaxRanks];
  if (threadIdx.x < nr) base[threadIdx.x] = resolve(pt, threadIdx.x, codes[0][threadIdx.x]);
  __syncthreads();
  // one descriptor per peer (uniform base, per-lane 32-bit offsets: host checks < 4 GiB)
  Rsrc src[NRM];
#pragma unroll
  for (int j = 0; j < NRM; ++j)
    if (j < nr) src[j] = make_rsrc(uniform_ptr(const_cast<char*>(base[j])), 0xFFFFFFF0u);
  for (uint64_t idx = r.lo + threadIdx.x; idx < r.hi; idx += kThreads) {
    const uint64_t m = idx / rowv, v = idx % rowv;
    u32x4 x[NRM];
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr) x[j] = ld16(src[j], (uint32_t)((m * rowv + v) * 16));
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr) *reinterpret_cast<u32x4*>(a.out + ((m * nr + j) * rowv + v) * 16) = x[j];
    } else {
#pragma unroll
      for (int j = 0; j < NRM; ++j)
        if (j < nr) x[j] = ld16(src[j], (uint32_t)(((m * nr + me) * rowv + v) * 16));
      VecAcc<DT> acc;
      acc.load(x[0]);
#pragma unroll
      for (int j = 1; j < NRM; ++j)
        if (j < nr) acc.template acc<OP>(x[j]);
      *reinterpret_cast<u32x4*>(a.out + (m * rowv + v) * 16) = acc.store();
    }
  }
  if (!sync_phase(a, 3, e)) return;
  finish(a, e);
}

// Local element-wise reduction: out = op(in0, in1, ...) for the fused
// last-axis reduce-scatter and the P2P ring/RHD schedules.
template <int DT, int OP>
__global__ void __launch_bounds__(kThreads) k_local_reduce(LocalReduceArgs a) {
  // vectors grid-strided; each input pointer must be 16-B aligned
  const uint64_t nv = a.nbytes / 16;
  for (uint64_t v = (uint64_t)blockIdx.x * kThreads + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * kThreads) {
    VecAcc<DT> acc;
    acc.load(*reinterpret_cast<const u32x4*>(a.in[0] + v * 16));
    for (int j = 1; j < a.n_in; ++j) acc.template acc<OP>(*reinterpret_cast<const u32x4*>(a.in[j] + v * 16));
    *reinterpret_cast<u32x4*>(a.out + v * 16) = acc.store();
  }
  const uint64_t tail = a.nbytes - nv * 16;
  if (tail && blockIdx.x == 0 && threadIdx.x == 0) {
    using E = Elem<DT>;
    for (uint32_t o = 0; o < tail; o += E::B) {
      typename E::A acc = E::ld(make_rsrc(a.in[0] + nv * 16, (uint32_t)tail), o);
      for (int j = 1; j < a.n_in; ++j) acc = apply_op<OP>(acc, E::ld(make_rsrc(a.in[j] + nv * 16, (uint32_t)tail), o));
      E::st(make_rsrc(a.out + nv * 16, (uint32_t)tail), o, acc);
    }
  }
}

// Streaming device copy (single-rank "all-reduce" and staging): 16-B
// non-temporal loads/stores; one contiguous 4 KiB slice per workgroup
// (CONTIG) or a grid-stride loop with U vectors in flight per lane.  The
// round-1 sweep of 13 (U, LNT, SNT, CONTIG) variants is in profiles/r1_copy;
// only the measured winner is instantiated (launch_copy).
template <int U, bool LNT, bool SNT, bool CONTIG>
__global__ void __launch_bounds__(kThreads) k_copy_v(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t nv) {
  uint64_t v, stride, end;
  if (CONTIG) {
    const uint64_t per = ((nv + gridDim.x - 1) / gridDim.x + kThreads - 1) / kThreads * kThreads;
    v = (uint64_t)blockIdx.x * per + threadIdx.x;
    end = std::min<uint64_t>(nv, (uint64_t)(blockIdx.x + 1) * per);
    stride = kThreads;
  } else {
    v = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    end = nv;
    stride = (uint64_t)gridDim.x * kThreads;
  }
  for (; v + (U - 1) * stride < end; v += U * stride) {
    u32x4 r[U];
#pragma unroll
    for (int i = 0; i < U; ++i) r[i] = LNT ? __builtin_nontemporal_load(src + v + i * stride) : src[v + i * stride];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (SNT) __builtin_nontemporal_store(r[i], dst + v + i * stride);
      else dst[v + i * stride] = r[i];
    }
  }
  for (; v < end; v += stride) dst[v] = src[v];
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
void launch_copy(const void* src, void* dst, uint64_t nbytes, hipStream_t s) {
  if (nbytes == 0 || src == dst) return;
  const uint64_t a = (uint64_t)src | (uint64_t)dst;
  if (a % 16 || nbytes < (1u << 20)) {
    CCMPI_HIP_CHECK(hipMemcpyAsync(dst, src, nbytes, hipMemcpyDeviceToDevice, s));
    return;
  }
  // One contiguous 4 KiB slice per workgroup (one 16-B non-temporal vector per
  // lane) up to 2^20 workgroups, longer slices beyond.  Measured on MI355X
  // (profiles/r1_copy): 3.1-3.2 TB/s algbw at 1 GiB vs 2.4-2.6 for the runtime
  // blit and 2.2-2.5 for a grid-stride loop, which interleaves every
  // workgroup's accesses over the whole buffer.
  const uint64_t nv = nbytes / 16;
  const int grid = (int)std::min<uint64_t>((nv + kThreads - 1) / kThreads, 1u << 20);
  hipLaunchKernelGGL((k_copy_v<1, true, true, true>), dim3(grid), dim3(kThreads), 0, s, (const u32x4*)src, (u32x4*)dst,
                     nv);
  CCMPI_HIP_CHECK(hipGetLastError());
  if (nbytes % 16)
    CCMPI_HIP_CHECK(hipMemcpyAsync((char*)dst + nv * 16, (const char*)src + nv * 16, nbytes % 16,
                                   hipMemcpyDeviceToDevice, s));
}

int grid_for(uint64_t bytes_per_cta_work, int max_blocks) {
  // at least kCtaBytes (CCMPI_CTA_BYTES, default 64 KiB) of work per CTA; at most max_blocks CTAs
  static const uint64_t kCtaBytes = [] {
    const char* e = std::getenv("CCMPI_CTA_BYTES");
    const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
    return v >= 4096 ? v : (uint64_t)(64u << 10);
  }();
  uint64_t g = (bytes_per_cta_work + kCtaBytes - 1) / kCtaBytes;
  if (g < 1) g = 1;
  if (g > (uint64_t)max_blocks) g = max_blocks;
  if (g > (uint64_t)kMaxBlocks) g = kMaxBlocks;
  return (int)g;
}

template <typename F>
static void with_nrm(int nranks, F&& f) {
  if (nranks <= 8) f.template operator()<8>();
  else if (nranks <= kMaxRanks) f.template operator()<kMaxRanks>();
  else throw std::invalid_argument("ccmpi: too many ranks for the device communicator");
}

void launch_allreduce(int algo, const CollArgs& a, int nranks, int dtype, int op, int grid, hipStream_t s) {
  with_nrm(nranks, [&]<int R>() {
    dispatch_dt_op(dtype, op, [&]<int D, int O>() {
      switch (algo) {
        case ALGO_ONESHOT: hipLaunchKernelGGL((k_allreduce_oneshot<D, O, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_TWOSHOT: hipLaunchKernelGGL((k_allreduce_twoshot<D, O, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_REDUCE_BCAST: hipLaunchKernelGGL((k_allreduce_reduce_bcast<D, O, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_TWOSHOT_PUSH: hipLaunchKernelGGL((k_allreduce_twoshot_push<D, O, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_RING: hipLaunchKernelGGL((k_allreduce_ring<D, O>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_RHD: hipLaunchKernelGGL((k_allreduce_rhd<D, O>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_LL: hipLaunchKernelGGL((k_allreduce_ll<D, O>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_TWOSHOT_FANOUT: hipLaunchKernelGGL((k_allreduce_twoshot_fanout<D, O, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
        case ALGO_TWOSHOT_FANOUT_LDS:
          hipLaunchKernelGGL((k_allreduce_twoshot_fanout<D, O, R, true>), dim3(grid), dim3(kThreads), 0, s, a);
          break;
        default: throw std::invalid_argument("ccmpi: bad allreduce algo");
      }
    });
  });
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_inbox_to_local(const CollArgs& a, int nranks, int dtype, int grid, hipStream_t s) {
  with_nrm(nranks, [&]<int R>() {
    if (dtype == DT_BF16) hipLaunchKernelGGL((k_allreduce_inbox_local<DT_BF16, OP_SUM, R>), dim3(grid), dim3(kThreads), 0, s, a);
    else if (dtype == DT_F32) hipLaunchKernelGGL((k_allreduce_inbox_local<DT_F32, OP_SUM, R>), dim3(grid), dim3(kThreads), 0, s, a);
    else throw std::invalid_argument("ccmpi: inbox all-reduce supports bf16 / fp32 sums");
  });
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_inbox_mean(const CollArgs& a, int nranks, int grid, hipStream_t s) {
  with_nrm(nranks, [&]<int R>() { hipLaunchKernelGGL((k_inbox_mean<R>), dim3(grid), dim3(kThreads), 0, s, a); });
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_reduce_scatter(const CollArgs& a, int nranks, int dtype, int op, int grid, hipStream_t s) {
  with_nrm(nranks, [&]<int R>() {
    dispatch_dt_op(dtype, op, [&]<int D, int O>() {
      hipLaunchKernelGGL((k_reduce_scatter<D, O, R>), dim3(grid), dim3(kThreads), 0, s, a);
    });
  });
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_lastaxis(int mode, const CollArgs& a, int nranks, int dtype, int op, int grid, hipStream_t s) {
  with_nrm(nranks, [&]<int R>() {
    if (mode == 0) {
      hipLaunchKernelGGL((k_lastaxis<0, DT_F32, OP_SUM, R>), dim3(grid), dim3(kThreads), 0, s, a);
    } else {
      dispatch_dt_op(dtype, op, [&]<int D, int O>() {
        hipLaunchKernelGGL((k_lastaxis<1, D, O, R>), dim3(grid), dim3(kThreads), 0, s, a);
      });
    }
  });
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_move(int mode, const CollArgs& a, int nranks, int grid, hipStream_t s) {
  with_nrm(nranks, [&]<int R>() {
    switch (mode) {
      case MOVE_ALLGATHER: hipLaunchKernelGGL((k_move<0, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
      case MOVE_ALLTOALL: hipLaunchKernelGGL((k_move<1, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
      case MOVE_BCAST: hipLaunchKernelGGL((k_move<2, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
      case MOVE_ALLTOALL_PUSH: hipLaunchKernelGGL((k_move<3, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
      case MOVE_ALLGATHER_PUSH: hipLaunchKernelGGL((k_move<4, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
      case MOVE_BCAST_PUSH: hipLaunchKernelGGL((k_move<5, R>), dim3(grid), dim3(kThreads), 0, s, a); break;
      default: throw std::invalid_argument("ccmpi: bad move mode");
    }
  });
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_alltoall_pairwise(const CollArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_alltoall_pairwise, dim3(grid), dim3(kThreads), 0, s, a);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_alltoallv(const VArgs& v, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_alltoallv_push, dim3(grid), dim3(kThreads), 0, s, v);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_alltoallv_dev(const VDevArgs& v, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_alltoallv_dev, dim3(grid), dim3(kThreads), 0, s, v);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void launch_local_reduce(const LocalReduceArgs& a, int dtype, int op, hipStream_t s) {
  uint64_t nv = a.nbytes / 16;
  int grid = (int)std::min<uint64_t>(std::max<uint64_t>((nv + kThreads - 1) / kThreads, 1), 2048);
  dispatch_dt_op(dtype, op, [&]<int D, int O>() {
    hipLaunchKernelGGL((k_local_reduce<D, O>), dim3(grid), dim3(kThreads), 0, s, a);
  });
  CCMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace dev
}  // namespace ccmpi
