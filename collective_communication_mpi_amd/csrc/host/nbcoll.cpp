// Non-blocking collectives of the host plane (MPI-3 Ibarrier / Ibcast /
// Iallreduce / Iallgather / Ialltoall / Ireduce_scatter_block).
//
// The reference only reaches non-blocking communication through Isend/Irecv +
// Waitall in myAlltoall (mpi_wrapper/comm.py:130-155) and argues for it in its
// README (README.md:145: overlap / pipelining).  Here every collective of that
// family can be started and overlapped with local work:
//
//   * a collective is a schedule of ROUNDS; round k posts its irecvs/isends on
//     the P2P rings with the internal tag (base - k), and its local work
//     (a reduction of what arrived) runs once every message of the round
//     completed, then round k+1 is posted;
//   * every started collective is held by the communicator until it finished,
//     and EVERY progress() call (any Wait/Test/blocking P2P on this comm)
//     advances them: a rank blocked in an unrelated receive still forwards its
//     ring neighbours' chunks, so non-blocking collectives never wait for the
//     owner's Wait to make progress;
//   * each started collective takes a fresh tag base from a per-comm sequence
//     (every rank starts collectives in the same order), so any number can be
//     in flight together and with user P2P traffic (negative tags never match
//     ANY_TAG receives).
//
// Schedules: dissemination barrier (ceil(log2 p) rounds), binomial-tree bcast,
// all-reduce as one all-pairs round + rank-order reduction for small buffers
// (bitwise identical on every rank) or ring reduce-scatter + all-gather for
// large ones, all-pairs all-gather / all-to-all (one round), ring
// reduce-scatter (p-1 rounds).
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "shm_comm.hpp"

namespace ccmpi {

namespace {

constexpr int kTagNbBase = -(1 << 20);
constexpr int kNbStride = 1024;   // rounds per collective (tags base .. base-1023)
constexpr int kNbSlots = 1 << 16; // distinct tag bases before reuse
constexpr size_t kSmallAllreduce = 16 << 10;  // all-pairs all-reduce up to this many bytes

int mod(int a, int p) { return ((a % p) + p) % p; }

bool overlaps(const void* a, size_t na, const void* b, size_t nb) {
  const char* x = static_cast<const char*>(a);
  const char* y = static_cast<const char*>(b);
  return na && nb && x < y + nb && y < x + na;
}

}  // namespace

void NbColl::recv(ShmComm& c, void* b, size_t n, int src, int k) { reqs.push_back(c.irecv(b, n, src, tag - k)); }

void NbColl::send(ShmComm& c, const void* b, size_t n, int dst, int k) {
  reqs.push_back(c.isend_internal(b, n, dst, tag - k));
}

namespace {

// Dissemination barrier: round k signals rank r + 2^k and waits for r - 2^k.
struct NbBarrier final : NbColl {
  int p, r;
  char tok[2] = {0, 0};
  NbBarrier(int p_, int r_) : p(p_), r(r_) {}
  bool post(ShmComm& c, int k) override {
    if (k >= 31 || (1 << k) >= p) return false;
    const int d = 1 << k;
    recv(c, &tok[1], 1, mod(r - d, p), k);
    send(c, &tok[0], 1, mod(r + d, p), k);
    return true;
  }
};

// Binomial tree rooted at `root` (ranks relative to the root): receive from the
// parent (vr minus its lowest set bit), then send to every child vr + 2^j,
// 2^j < lowbit(vr), all at once.
struct NbBcast final : NbColl {
  char* buf;
  size_t nb;
  int p, r, root;
  NbBcast(char* b, size_t n, int p_, int r_, int root_) : buf(b), nb(n), p(p_), r(r_), root(root_) {}
  bool post(ShmComm& c, int k) override {
    const int vr = mod(r - root, p);
    const int low = vr ? (vr & -vr) : (1 << 30);
    if (k == 0) {
      if (vr) recv(c, buf, nb, mod(vr - low + root, p), 0);
      return true;
    }
    if (k == 1) {
      // tag offset 0: the child receives this in ITS round 0
      for (int m = 1; m < low && vr + m < p; m <<= 1) send(c, buf, nb, mod(vr + m + root, p), 0);
      return true;
    }
    return false;
  }
};

// Small all-reduce: one round in which every rank sends its whole buffer to
// every peer; then dst = x_0 op x_1 op ... op x_{p-1} in rank order.
struct NbAllreducePairs final : NbColl {
  char* dst;
  size_t count, nb;
  int dt, op, p, r;
  NbAllreducePairs(const void* src, char* d, size_t cnt, int dt_, int op_, int p_, int r_)
      : dst(d), count(cnt), nb(cnt * dtype_size(dt_)), dt(dt_), op(op_), p(p_), r(r_) {
    tmp.resize(nb * (size_t)p);
    std::memcpy(tmp.data() + nb * (size_t)r, src ? src : d, nb);
  }
  bool post(ShmComm& c, int k) override {
    if (k) return false;
    for (int i = 0; i < p; ++i)
      if (i != r) recv(c, tmp.data() + nb * (size_t)i, nb, i, 0);
    for (int i = 0; i < p; ++i)
      if (i != r) send(c, tmp.data() + nb * (size_t)r, nb, i, 0);
    return true;
  }
  void finish(int) override {
    std::memcpy(dst, tmp.data(), nb);
    for (int i = 1; i < p; ++i) reduce_inplace(dst, tmp.data() + nb * (size_t)i, count, dt, op);
  }
};

// Chunk c of a `count`-element buffer split in p near-equal parts.
struct Chunks {
  size_t count;
  int p;
  size_t lo(int c) const { return count * (size_t)mod(c, p) / (size_t)p; }
  size_t len(int c) const { return count * (size_t)(mod(c, p) + 1) / (size_t)p - lo(c); }
};

// Large all-reduce: ring reduce-scatter (rounds 0..p-2: send chunk r-k, reduce
// the incoming chunk r-k-1) then ring all-gather (rounds p-1..2p-3: forward the
// owned sums, received straight into place).
struct NbAllreduceRing final : NbColl {
  char* d;
  Chunks ch;
  size_t es;
  int dt, op, p, r;
  NbAllreduceRing(const void* src, char* dst, size_t cnt, int dt_, int op_, int p_, int r_)
      : d(dst), ch{cnt, p_}, es(dtype_size(dt_)), dt(dt_), op(op_), p(p_), r(r_) {
    if (src && src != dst) std::memmove(d, src, cnt * es);
    tmp.resize((cnt / (size_t)p + 1) * es);
  }
  bool post(ShmComm& c, int k) override {
    const int right = mod(r + 1, p), left = mod(r - 1, p);
    if (k < p - 1) {
      recv(c, tmp.data(), ch.len(r - k - 1) * es, left, k);
      send(c, d + ch.lo(r - k) * es, ch.len(r - k) * es, right, k);
      return true;
    }
    if (k < 2 * (p - 1)) {
      const int s = k - (p - 1);
      recv(c, d + ch.lo(r - s) * es, ch.len(r - s) * es, left, k);
      send(c, d + ch.lo(r + 1 - s) * es, ch.len(r + 1 - s) * es, right, k);
      return true;
    }
    return false;
  }
  void finish(int k) override {
    if (k < p - 1) reduce_inplace(d + ch.lo(r - k - 1) * es, tmp.data(), ch.len(r - k - 1), dt, op);
  }
};

// All-gather / all-to-all: one round, every peer's block in flight at once.
struct NbAllgather final : NbColl {
  const char* mine;
  char* dst;
  size_t nb;
  int p, r;
  NbAllgather(const void* src, char* d, size_t n, int p_, int r_) : dst(d), nb(n), p(p_), r(r_) {
    char* own = d + nb * (size_t)r;
    if (src && src != own) {
      if (overlaps(src, nb, d, nb * (size_t)p)) {
        tmp.assign(static_cast<const char*>(src), static_cast<const char*>(src) + nb);
        src = tmp.data();
      }
      std::memmove(own, src, nb);
    }
    mine = own;
  }
  bool post(ShmComm& c, int k) override {
    if (k) return false;
    for (int i = 0; i < p; ++i)
      if (i != r) recv(c, dst + nb * (size_t)i, nb, i, 0);
    for (int i = 0; i < p; ++i)
      if (i != r) send(c, mine, nb, i, 0);
    return true;
  }
};

struct NbAlltoall final : NbColl {
  const char* s;
  char* dst;
  size_t blk;
  int p, r;
  NbAlltoall(const void* src, char* d, size_t b, int p_, int r_) : dst(d), blk(b), p(p_), r(r_) {
    const size_t total = blk * (size_t)p;
    s = src ? static_cast<const char*>(src) : d;
    if (overlaps(s, total, d, total)) {  // in place: send from a private copy
      tmp.assign(s, s + total);
      s = tmp.data();
    }
    std::memmove(d + blk * (size_t)r, s + blk * (size_t)r, blk);
  }
  bool post(ShmComm& c, int k) override {
    if (k) return false;
    for (int i = 0; i < p; ++i)
      if (i != r) recv(c, dst + blk * (size_t)i, blk, i, 0);
    for (int i = 0; i < p; ++i)
      if (i != r) send(c, s + blk * (size_t)i, blk, i, 0);
    return true;
  }
};

// Ring reduce-scatter ending with block r on rank r: round k sends the partial
// of block r-k-1 to the right and reduces the left's partial of block r-k-2.
struct NbReduceScatter final : NbColl {
  char* dst;
  size_t count, nb;
  int dt, op, p, r;
  NbReduceScatter(const void* src, char* d, size_t cnt, int dt_, int op_, int p_, int r_)
      : dst(d), count(cnt), nb(cnt * dtype_size(dt_)), dt(dt_), op(op_), p(p_), r(r_) {
    tmp.resize(nb * (size_t)(p + 1));  // p working blocks + one receive block
    std::memcpy(tmp.data(), src ? src : d, nb * (size_t)p);
    if (p == 1) std::memcpy(dst, tmp.data(), nb);
  }
  char* blk(int b) { return tmp.data() + nb * (size_t)mod(b, p); }
  bool post(ShmComm& c, int k) override {
    if (k >= p - 1) return false;
    recv(c, tmp.data() + nb * (size_t)p, nb, mod(r - 1, p), k);
    send(c, blk(r - k - 1), nb, mod(r + 1, p), k);
    return true;
  }
  void finish(int k) override {
    reduce_inplace(blk(r - k - 2), tmp.data() + nb * (size_t)p, count, dt, op);
    if (k == p - 2) std::memcpy(dst, blk(r), nb);
  }
};

}  // namespace

RequestPtr ShmComm::isend_internal(const void* buf, size_t nbytes, int dest, int tag) {
  if (tag >= 0) throw std::invalid_argument("ccmpi: internal tags are negative");
  return isend_raw(buf, nbytes, dest, tag);
}

NbCollPtr ShmComm::nb_start_(NbCollPtr c) {
  if (size_ * 2 > kNbStride) throw std::invalid_argument("ccmpi: non-blocking collectives support <= 512 ranks");
  c->tag = kTagNbBase - (int)(nb_seq_++ % (uint64_t)kNbSlots) * kNbStride;
  nb_active_.push_back(c);
  nb_progress_();  // posts round 0 (guarded: posting may re-enter progress())
  return c;
}

bool ShmComm::nb_advance_(NbColl& c) {
  while (!c.done) {
    for (auto& r : c.reqs)
      if (!r->complete) return false;
    for (auto& r : c.reqs)
      if (r->truncated && c.err.empty()) c.err = "ccmpi: non-blocking collective message truncated (buffer sizes differ across ranks)";
    if (c.round >= 0) c.finish(c.round);
    c.reqs.clear();
    ++c.round;
    if (!c.post(*this, c.round)) c.done = true;
  }
  return true;
}

void ShmComm::nb_progress_() {
  if (nb_in_progress_) return;  // posting a round may progress() again
  nb_in_progress_ = true;
  try {
    for (size_t i = 0; i < nb_active_.size(); ++i) nb_advance_(*nb_active_[i]);
  } catch (...) {
    nb_in_progress_ = false;
    throw;
  }
  nb_active_.erase(std::remove_if(nb_active_.begin(), nb_active_.end(),
                                  [](const NbCollPtr& c) { return c->done; }),
                   nb_active_.end());
  nb_in_progress_ = false;
}

bool ShmComm::nb_test(const NbCollPtr& c) {
  if (!c->done) {
    progress();
    nb_progress_();
  }
  if (c->done && !c->err.empty()) throw std::runtime_error(c->err);
  return c->done;
}

void ShmComm::nb_wait(const NbCollPtr& c) {
  uint64_t spins = 0;
  double t0 = wtime();
  while (!c->done) {
    bool moved = progress();
    nb_progress_();
    if (!moved) backoff_(spins);
    else spins = 0;
    if ((++spins & 1023) == 0 && wtime() - t0 > timeout_s_) timeout_("non-blocking collective");
  }
  if (!c->err.empty()) throw std::runtime_error(c->err);
}

NbCollPtr ShmComm::ibarrier() { return nb_start_(std::make_shared<NbBarrier>(size_, rank_)); }

NbCollPtr ShmComm::ibcast(void* buf, size_t nbytes, int root) {
  if (root < 0 || root >= size_) throw std::invalid_argument("ccmpi: invalid root");
  return nb_start_(std::make_shared<NbBcast>(static_cast<char*>(buf), nbytes, size_, rank_, root));
}

NbCollPtr ShmComm::iallreduce(const void* sbuf, void* rbuf, size_t count, int dt, int op) {
  if (!reduce_supported(dt, op)) throw std::invalid_argument("ccmpi: unsupported reduction for Iallreduce");
  char* d = static_cast<char*>(rbuf);
  if (count * dtype_size(dt) <= kSmallAllreduce || count < (size_t)size_)
    return nb_start_(std::make_shared<NbAllreducePairs>(sbuf, d, count, dt, op, size_, rank_));
  return nb_start_(std::make_shared<NbAllreduceRing>(sbuf, d, count, dt, op, size_, rank_));
}

NbCollPtr ShmComm::iallgather(const void* sbuf, size_t nbytes, void* rbuf) {
  return nb_start_(std::make_shared<NbAllgather>(sbuf, static_cast<char*>(rbuf), nbytes, size_, rank_));
}

NbCollPtr ShmComm::ialltoall(const void* sbuf, size_t block_bytes, void* rbuf) {
  return nb_start_(std::make_shared<NbAlltoall>(sbuf, static_cast<char*>(rbuf), block_bytes, size_, rank_));
}

NbCollPtr ShmComm::ireduce_scatter_block(const void* sbuf, void* rbuf, size_t count, int dt, int op) {
  if (!reduce_supported(dt, op)) throw std::invalid_argument("ccmpi: unsupported reduction for Ireduce_scatter_block");
  return nb_start_(std::make_shared<NbReduceScatter>(sbuf, static_cast<char*>(rbuf), count, dt, op, size_, rank_));
}

}  // namespace ccmpi
