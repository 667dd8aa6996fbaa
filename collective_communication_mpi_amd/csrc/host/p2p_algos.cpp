// The reference's hand-written collectives, run as native P2P schedules on the
// host plane's message rings.  The message pattern is the reference's own
// (mpi_wrapper/comm.py); only the per-message cost changes: no Python frame,
// no buffer-spec parsing and no NumPy ufunc dispatch between messages.
//
//   my_reduce_bcast       comm.py:63-107   rank 0 receives rank 1..p-1 in order,
//                                          reduces each into dst, then sends dst
//                                          back to 1..p-1 in order
//   my_alltoall_nb        comm.py:110-159  own block copied, all irecvs posted,
//                                          then all isends, waitall
//   my_alltoall_pairwise  comm.py:162-199  for i in 0..p-1: sendrecv with rank i
//   my_ring_allreduce     ring reduce-scatter + all-gather (2(p-1) steps)
//   my_rhd_allreduce      recursive halving / doubling (power-of-two p)
//
// Messages carry negative internal tags, so user receives posted with
// ANY_TAG never match them (tag_match in shm_comm.cpp).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "shm_comm.hpp"

namespace ccmpi {

namespace {

constexpr int kTagReduceBcast = -16;
constexpr int kTagAlltoall = -17;
constexpr int kTagPairwise = -18;
constexpr int kTagRing = -19;   // ring steps use kTagRing - step (one tag per step)
constexpr int kTagRhd = -4096;  // rhd rounds use kTagRhd - round
// reduce_bcast root: pre-post every receive (p scratch slices) up to this many bytes
constexpr size_t kPrepostMaxBytes = size_t(4) << 20;

// per-thread scratch, grown on demand (the schedules run with the GIL released)
char* scratch(size_t nbytes) {
  thread_local std::vector<char> buf;
  if (buf.size() < nbytes) buf.resize(std::max(nbytes, (size_t)4096));
  return buf.data();
}

// Touch every page of [p, p + n) with a write (the bytes written are overwritten by the
// result afterwards).  A freshly allocated result buffer faults on first touch (~2-5 us
// per page with the zero fill); doing that while this rank idles waiting for a peer
// keeps the fault off the schedule's critical path.
void prefault(void* p, size_t n) {
  constexpr uintptr_t kPage = 4096;
  volatile char* c = static_cast<volatile char*>(p);
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  for (uintptr_t o = 0; o < n; o = ((a + o) / kPage + 1) * kPage - a) c[o] = 0;
}

}  // namespace

// Optional phase timestamps of the reduce->bcast schedule (CCMPI_P2P_TRACE=1), read back
// with p2p_trace(): a diagnostic for where a call's time goes, off by default.
// The buffer is shared by every thread of the process (schedules run with the GIL
// released), so it is guarded, and capped: nobody has to read it.
// CCMPI_P2P_TRACE=2 adds marks inside isend_raw (shm_comm.cpp): entry, request allocated,
// queued, payload copied into the peer's ring and published.
bool g_p2p_trace_on = std::getenv("CCMPI_P2P_TRACE") != nullptr;
bool g_p2p_trace_fine = g_p2p_trace_on && std::atoi(std::getenv("CCMPI_P2P_TRACE")) >= 2;

namespace {

constexpr size_t kTraceCap = size_t(1) << 20;
std::mutex g_trace_mu;
std::vector<double> g_trace;

inline void trace_mark() {
  if (!g_p2p_trace_on) return;
  const double t = wtime();
  std::lock_guard<std::mutex> lk(g_trace_mu);
  if (g_trace.size() < kTraceCap) g_trace.push_back(t);
}

bool overlaps(const void* a, const void* b, size_t n) {
  const char* x = static_cast<const char*>(a);
  const char* y = static_cast<const char*>(b);
  return n && x < y + n && y < x + n;
}

}  // namespace

void p2p_trace_mark() { trace_mark(); }

std::vector<double> p2p_trace_take() {
  std::vector<double> v;
  std::lock_guard<std::mutex> lk(g_trace_mu);
  v.swap(g_trace);
  return v;
}

void ShmComm::my_reduce_bcast(const void* src, void* dst, size_t count, int dt, int op) {
  if (!reduce_supported(dt, op)) throw std::invalid_argument("ccmpi: unsupported reduction for myAllreduce");
  const size_t nb = count * dtype_size(dt);
  if (rank_ == 0) {
    // every receive is posted before the first wait, each into its own scratch slice, so
    // the contributions land in place as they arrive (a receive posted late finds the
    // message in the unexpected queue: a heap copy, then a second copy); the reduction
    // still runs in rank order 1..p-1, as in the reference
    if (nb * (size_t)size_ > kPrepostMaxBytes) {  // large: one scratch slice, receives in turn
      if (dst != src) std::memmove(dst, src, nb);
      char* tmp = scratch(nb);
      for (int i = 1; i < size_; ++i) {
        recv(tmp, nb, i, kTagReduceBcast);
        reduce_inplace(dst, tmp, count, dt, op);
      }
      std::vector<RequestPtr> rs;
      rs.reserve(size_);
      for (int i = 1; i < size_; ++i) rs.push_back(isend_raw(dst, nb, i, kTagReduceBcast));
      waitall(rs);
      return;
    }
    // slices 1..p-1 receive, slice 0 accumulates: the sends go out of scratch and the copy
    // into dst (whose first touch may fault) comes after them
    trace_mark();
    char* tmp = scratch(nb * (size_t)size_);
    char* acc = tmp;
    std::vector<RequestPtr> rr;
    rr.reserve(size_);
    for (int i = 1; i < size_; ++i) rr.push_back(irecv(tmp + nb * (size_t)i, nb, i, kTagReduceBcast));
    std::memcpy(acc, src, nb);
    trace_mark();
    for (int i = 1; i < size_; ++i) {
      wait(rr[i - 1]);
      trace_mark();
      reduce_inplace(acc, tmp + nb * (size_t)i, count, dt, op);
    }
    // the reference sends in rank order with blocking Sends; posting them all
    // and waiting once keeps that order on every ring and lets small results
    // leave without a round trip per peer
    std::vector<RequestPtr> rs;
    rs.reserve(size_);
    for (int i = 1; i < size_; ++i) rs.push_back(isend_raw(acc, nb, i, kTagReduceBcast));
    trace_mark();
    std::memmove(dst, acc, nb);
    waitall(rs);
    trace_mark();
  } else {
    if (overlaps(dst, src, nb)) {
      // any overlap (not only dst == src): the prefault below writes dst while a message
      // larger than the ring is still being pushed from src during wait(rs)
      char* tmp = scratch(nb);
      std::memcpy(tmp, src, nb);
      src = tmp;
    }
    trace_mark();
    auto rr = irecv(dst, nb, 0, kTagReduceBcast);  // posted first: the result lands in place
    trace_mark();
    auto rs = isend_raw(src, nb, 0, kTagReduceBcast);
    trace_mark();
    // no receive progress has run since the irecv (isend_raw only pushes the send), so
    // dst holds no result bytes yet: fault its pages in while the root reduces
    prefault(dst, nb);
    trace_mark();
    wait(rs);
    trace_mark();
    wait(rr);
    trace_mark();
  }
}

void ShmComm::my_alltoall_nb(const void* src, void* dst, size_t block_bytes) {
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  const size_t total = block_bytes * (size_t)size_;
  if (overlaps(s, d, total)) {  // in place: send from a private copy
    char* tmp = scratch(total);
    std::memcpy(tmp, s, total);
    s = tmp;
  }
  std::memcpy(d + (size_t)rank_ * block_bytes, s + (size_t)rank_ * block_bytes, block_bytes);
  std::vector<RequestPtr> rs;
  rs.reserve(2 * (size_t)size_);
  for (int i = 0; i < size_; ++i)
    if (i != rank_) rs.push_back(irecv(d + (size_t)i * block_bytes, block_bytes, i, kTagAlltoall));
  for (int i = 0; i < size_; ++i)
    if (i != rank_) rs.push_back(isend_raw(s + (size_t)i * block_bytes, block_bytes, i, kTagAlltoall));
  waitall(rs);
}

void ShmComm::my_alltoall_pairwise(const void* src, void* dst, size_t block_bytes) {
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  const size_t total = block_bytes * (size_t)size_;
  if (overlaps(s, d, total)) {
    char* tmp = scratch(total);
    std::memcpy(tmp, s, total);
    s = tmp;
  }
  for (int i = 0; i < size_; ++i) {
    char* out = d + (size_t)i * block_bytes;
    const char* in = s + (size_t)i * block_bytes;
    if (i == rank_) {
      std::memcpy(out, in, block_bytes);
    } else {
      auto rr = irecv(out, block_bytes, i, kTagPairwise);
      wait(isend_raw(in, block_bytes, i, kTagPairwise));
      wait(rr);
    }
  }
}

void ShmComm::my_ring_allreduce(const void* src, void* dst, size_t count, int dt, int op) {
  if (!reduce_supported(dt, op)) throw std::invalid_argument("ccmpi: unsupported reduction for ring all-reduce");
  const size_t es = dtype_size(dt);
  char* d = static_cast<char*>(dst);
  if (dst != src) std::memmove(d, src, count * es);
  const int p = size_;
  if (p == 1 || count == 0) return;
  auto lo = [&](int c) { c = ((c % p) + p) % p; return count * (size_t)c / (size_t)p; };
  auto len = [&](int c) { c = ((c % p) + p) % p; return count * (size_t)(c + 1) / (size_t)p - count * (size_t)c / (size_t)p; };
  const int right = (rank_ + 1) % p, left = (rank_ - 1 + p) % p;
  char* tmp = scratch((count / p + 1) * es);
  // reduce-scatter: after p-1 steps rank r owns the full sum of chunk r+1
  for (int step = 0; step < p - 1; ++step) {
    const int sc = rank_ - step, rc = rank_ - step - 1;
    auto rr = irecv(tmp, len(rc) * es, left, kTagRing - step);
    auto sr = isend_raw(d + lo(sc) * es, len(sc) * es, right, kTagRing - step);
    wait(rr);
    reduce_inplace(d + lo(rc) * es, tmp, len(rc), dt, op);
    wait(sr);
  }
  // all-gather: circulate the owned sums (received straight into place)
  for (int step = 0; step < p - 1; ++step) {
    const int sc = rank_ + 1 - step, rc = rank_ - step;
    const int tag = kTagRing - (p - 1) - step;
    auto rr = irecv(d + lo(rc) * es, len(rc) * es, left, tag);
    auto sr = isend_raw(d + lo(sc) * es, len(sc) * es, right, tag);
    wait(rr);
    wait(sr);
  }
}

void ShmComm::my_rhd_allreduce(const void* src, void* dst, size_t count, int dt, int op) {
  const int p = size_;
  if (p & (p - 1)) return my_ring_allreduce(src, dst, count, dt, op);
  if (!reduce_supported(dt, op)) throw std::invalid_argument("ccmpi: unsupported reduction for rhd all-reduce");
  const size_t es = dtype_size(dt);
  char* d = static_cast<char*>(dst);
  if (dst != src) std::memmove(d, src, count * es);
  if (p == 1 || count == 0) return;
  char* tmp = scratch((count / 2 + 1) * es);
  size_t lo = 0, hi = count;
  std::vector<std::pair<size_t, size_t>> hist;
  int round = 0;
  // recursive halving: exchange half of the current range with partner rank^mask
  for (int mask = p / 2; mask >= 1; mask /= 2, ++round) {
    const int partner = rank_ ^ mask;
    const size_t mid = lo + (hi - lo) / 2;
    size_t klo = lo, khi = mid, slo = mid, shi = hi;
    if (rank_ & mask) { klo = mid; khi = hi; slo = lo; shi = mid; }
    auto rr = irecv(tmp, (khi - klo) * es, partner, kTagRhd - round);
    auto sr = isend_raw(d + slo * es, (shi - slo) * es, partner, kTagRhd - round);
    wait(rr);
    reduce_inplace(d + klo * es, tmp, khi - klo, dt, op);
    wait(sr);
    hist.emplace_back(lo, hi);
    lo = klo;
    hi = khi;
  }
  // recursive doubling: give back the owned range, receive the partner's half
  for (int mask = 1; mask <= p / 2; mask *= 2, ++round) {
    const int partner = rank_ ^ mask;
    auto [plo, phi] = hist.back();
    hist.pop_back();
    size_t olo, ohi;
    if (lo == plo) { olo = hi; ohi = phi; } else { olo = plo; ohi = lo; }
    auto rr = irecv(d + olo * es, (ohi - olo) * es, partner, kTagRhd - round);
    auto sr = isend_raw(d + lo * es, (hi - lo) * es, partner, kTagRhd - round);
    wait(rr);
    wait(sr);
    lo = plo;
    hi = phi;
  }
}

}  // namespace ccmpi
