// Shared-memory communicator: see shm_comm.hpp for the design.
#include "shm_comm.hpp"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#if defined(__x86_64__)
#include <immintrin.h>
#define CCMPI_RELAX() _mm_pause()
#else
#define CCMPI_RELAX() do {} while (0)
#endif

namespace ccmpi {

// ---------------------------------------------------------------------------
// segment layout
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t kMagic = 0x43434d5049414d44ull;  // "CCMPIAMD"
constexpr size_t kHdr = 16;                         // P2P frame header bytes

struct alignas(64) SegHeader {
  uint64_t magic;
  uint32_t size;
  uint32_t pad0;
  uint64_t ring_bytes;
  uint64_t slot_bytes;
  uint64_t total_bytes;
  alignas(64) std::atomic<uint32_t> attached;
  alignas(64) std::atomic<uint64_t> bar_arrive;
  alignas(64) std::atomic<uint64_t> bar_release;
};

struct alignas(64) ChanCtl {
  std::atomic<uint64_t> head;  // written by the sender
  char pad0[56];
  std::atomic<uint64_t> tail;  // written by the receiver
  char pad1[56];
};

static_assert(sizeof(ChanCtl) == 128, "ChanCtl layout");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "need lock-free 64-bit atomics");

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

size_t pow2_floor(size_t x) {
  size_t p = 1;
  while (p * 2 <= x) p *= 2;
  return p;
}

size_t env_size(const char* name, size_t dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return (size_t)std::strtoull(v, nullptr, 10);
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

std::string hex64(uint64_t v) {
  char b[17];
  std::snprintf(b, sizeof(b), "%016llx", (unsigned long long)v);
  return b;
}

// start time (clock ticks since boot) of a pid: field 22 of /proc/<pid>/stat
std::string proc_start(pid_t pid) {
  std::ifstream f("/proc/" + std::to_string(pid) + "/stat");
  std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  auto rp = s.rfind(')');
  if (rp == std::string::npos) return "0";
  std::istringstream is(s.substr(rp + 2));
  std::string tok;
  for (int field = 3; field <= 22 && (is >> tok); ++field) {
    if (field == 22) return tok;
  }
  return "0";
}

const char* envs(const char* n) {
  const char* v = std::getenv(n);
  return (v && *v) ? v : nullptr;
}

}  // namespace

struct Segment {
  SegHeader hdr;
};

double wtime() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

std::string job_id_from_env() {
  if (const char* j = envs("CCMPI_JOBID")) return j;
  pid_t pp = getppid();
  std::string parent = std::to_string(pp) + "@" + proc_start(pp);
  std::string key;
  if (envs("TORCHELASTIC_RUN_ID") && envs("MASTER_PORT")) {
    key = std::string("torchrun|") + (envs("MASTER_ADDR") ? envs("MASTER_ADDR") : "") + ":" +
          envs("MASTER_PORT") + "|" + envs("TORCHELASTIC_RUN_ID") + "|" +
          (envs("TORCHELASTIC_RESTART_COUNT") ? envs("TORCHELASTIC_RESTART_COUNT") : "0") +
          "|" + parent;
  } else if (envs("PMI_RANK") || envs("OMPI_COMM_WORLD_RANK")) {
    key = "pmi|" + parent;
  } else if (envs("MASTER_PORT")) {
    key = std::string("env|") + (envs("MASTER_ADDR") ? envs("MASTER_ADDR") : "") + ":" +
          envs("MASTER_PORT");
  } else {
    key = "ppid|" + parent;
  }
  return hex64(fnv1a(key));
}

// ---------------------------------------------------------------------------
// construction / attach
// ---------------------------------------------------------------------------
namespace {

size_t ring_bytes_for(int p) {
  size_t d = pow2_floor(std::max<size_t>(1, (32ull << 20) / ((size_t)p * p)));
  d = std::min<size_t>(std::max<size_t>(d, 16 << 10), 1 << 20);
  size_t e = env_size("CCMPI_RING_BYTES", d);
  return std::max<size_t>(pow2_floor(e), 4096);
}

size_t slot_bytes_for(int p) {
  size_t d = (64ull << 20) / ((size_t)p + 1);
  d = std::min<size_t>(std::max<size_t>(d, 256 << 10), 8 << 20);
  size_t e = env_size("CCMPI_SLOT_BYTES", d);
  return std::max<size_t>(round_up(e, 64), 4096);
}

struct Layout {
  size_t chan_off, flag_off, small_off, ring_off, slot_off, result_off, total;
};

// per-rank epoch flag (own cache line; written only by its rank)
struct alignas(64) EpochFlag {
  std::atomic<uint64_t> epoch;
  char pad[56];
};
static_assert(sizeof(EpochFlag) == 64, "EpochFlag layout");

// single-sync small-message collectives: per rank two (double-buffered by
// epoch parity) regions of kSmallBytes
constexpr size_t kSmallBytes = 8192;

Layout layout_for(int p, size_t ring, size_t slot) {
  Layout L;
  L.chan_off = round_up(sizeof(SegHeader), 128);
  L.flag_off = round_up(L.chan_off + sizeof(ChanCtl) * (size_t)p * p, 128);
  L.small_off = round_up(L.flag_off + sizeof(EpochFlag) * (size_t)p, 4096);
  L.ring_off = round_up(L.small_off + 2 * kSmallBytes * (size_t)p, 4096);
  L.slot_off = round_up(L.ring_off + ring * (size_t)p * p, 4096);
  L.result_off = L.slot_off + slot * (size_t)p;
  L.total = round_up(L.result_off + slot, 4096);
  return L;
}

}  // namespace

ShmComm::ShmComm(const std::string& name, int rank, int size)
    : name_(name), rank_(rank), size_(size) {
  if (size < 1 || rank < 0 || rank >= size)
    throw std::invalid_argument("ccmpi: bad rank/size");
  if (const char* t = envs("CCMPI_TIMEOUT")) timeout_s_ = std::atof(t);
  small_allreduce_max_ = std::min(env_size("CCMPI_SMALL_ALLREDUCE_BYTES", small_allreduce_max_), kSmallBytes);
  world_ranks_.resize(size);
  for (int i = 0; i < size; ++i) world_ranks_[i] = i;
  send_q_.resize(size);
  peer_tail_.assign(size, 0);
  unexpected_.resize(size);
  cur_.resize(size);
  attach_();
}

void ShmComm::attach_() {
  const size_t ring = ring_bytes_for(size_), slot = slot_bytes_for(size_);
  Layout L = layout_for(size_, ring, slot);
  std::string shm_name = "/" + name_;
  int fd = shm_open(shm_name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("ccmpi: shm_open(" + shm_name + ") failed: " + std::strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); throw std::runtime_error("ccmpi: fstat failed"); }
  if ((size_t)st.st_size < L.total) {
    if (ftruncate(fd, (off_t)L.total) != 0) {
      close(fd);
      throw std::runtime_error(std::string("ccmpi: ftruncate failed: ") + std::strerror(errno));
    }
  }
  void* p = mmap(nullptr, L.total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error(std::string("ccmpi: mmap failed: ") + std::strerror(errno));
  seg_ = static_cast<Segment*>(p);
  seg_bytes_ = L.total;
  SegHeader& h = seg_->hdr;
  // The first arrival stamps the geometry; others check it.  Fresh pages are zero.
  uint32_t prev = h.attached.fetch_add(1, std::memory_order_acq_rel);
  if (prev == 0) {
    h.size = (uint32_t)size_;
    h.ring_bytes = ring;
    h.slot_bytes = slot;
    h.total_bytes = L.total;
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&h.magic)->store(kMagic, std::memory_order_release);
  } else if (prev >= (uint32_t)size_) {
    throw std::runtime_error("ccmpi: stale shared segment " + shm_name +
                             " (more attaches than ranks); set CCMPI_JOBID to a fresh value");
  }
  uint64_t spins = 0;
  double t0 = wtime();
  while (reinterpret_cast<std::atomic<uint64_t>*>(&h.magic)->load(std::memory_order_acquire) != kMagic ||
         h.attached.load(std::memory_order_acquire) < (uint32_t)size_) {
    backoff_(spins);
    if ((spins & 1023) == 0 && wtime() - t0 > timeout_s_) timeout_("attach");
  }
  if (h.size != (uint32_t)size_ || h.ring_bytes != ring || h.slot_bytes != slot)
    throw std::runtime_error("ccmpi: segment geometry mismatch (CCMPI_RING_BYTES/CCMPI_SLOT_BYTES differ across ranks?)");
  if (rank_ == 0) shm_unlink(shm_name.c_str());
  // cache this rank's channel control blocks and rings (the progress engine
  // touches them on every poll)
  auto* ctl = reinterpret_cast<ChanCtl*>(reinterpret_cast<char*>(seg_) + L.chan_off);
  char* rings = reinterpret_cast<char*>(seg_) + L.ring_off;
  out_ctl_.resize(size_);
  in_ctl_.resize(size_);
  out_ring_.resize(size_);
  in_ring_.resize(size_);
  for (int j = 0; j < size_; ++j) {
    out_ctl_[j] = &ctl[(size_t)rank_ * size_ + j];
    in_ctl_[j] = &ctl[(size_t)j * size_ + rank_];
    out_ring_[j] = rings + ring * ((size_t)rank_ * size_ + j);
    in_ring_[j] = rings + ring * ((size_t)j * size_ + rank_);
  }
  ring_cap_ = ring;
  auto* flags = reinterpret_cast<EpochFlag*>(reinterpret_cast<char*>(seg_) + L.flag_off);
  flag_.resize(size_);
  for (int j = 0; j < size_; ++j) flag_[j] = &flags[j].epoch;
  small_base_ = reinterpret_cast<char*>(seg_) + L.small_off;
  slot_base_ = reinterpret_cast<char*>(seg_) + L.slot_off;
  result_base_ = reinterpret_cast<char*>(seg_) + L.result_off;
}

ShmComm::~ShmComm() {
  if (seg_) munmap(seg_, seg_bytes_);
}

std::shared_ptr<ShmComm> ShmComm::world() {
  int rank = 0, size = 1;
  auto geti = [](const char* a, const char* b, int* out) {
    const char* v = envs(a);
    if (!v && b) v = envs(b);
    if (v) { *out = std::atoi(v); return true; }
    return false;
  };
  bool have = false;
  if (envs("CCMPI_RANK") && envs("CCMPI_SIZE")) {
    geti("CCMPI_RANK", nullptr, &rank); geti("CCMPI_SIZE", nullptr, &size); have = true;
  } else if (envs("PMI_RANK") && envs("PMI_SIZE")) {
    geti("PMI_RANK", nullptr, &rank); geti("PMI_SIZE", nullptr, &size); have = true;
  } else if (envs("OMPI_COMM_WORLD_RANK") && envs("OMPI_COMM_WORLD_SIZE")) {
    geti("OMPI_COMM_WORLD_RANK", nullptr, &rank); geti("OMPI_COMM_WORLD_SIZE", nullptr, &size); have = true;
  } else if (envs("RANK") && envs("WORLD_SIZE")) {
    geti("RANK", nullptr, &rank); geti("WORLD_SIZE", nullptr, &size); have = true;
    if (const char* lws = envs("LOCAL_WORLD_SIZE")) {
      if (std::atoi(lws) != size)
        throw std::runtime_error("ccmpi: the shared-memory host plane is single-node; "
                                 "LOCAL_WORLD_SIZE != WORLD_SIZE");
    }
  }
  std::string job = have ? job_id_from_env() : ("solo" + std::to_string(getpid()) + "_" + proc_start(getpid()));
  if (!have) { rank = 0; size = 1; }
  return std::make_shared<ShmComm>("ccmpi_" + job + "_w", rank, size);
}

size_t ShmComm::slot_bytes() const { return seg_->hdr.slot_bytes; }
size_t ShmComm::ring_bytes() const { return seg_->hdr.ring_bytes; }

char* ShmComm::slot_(int r) { return slot_base_ + seg_->hdr.slot_bytes * (size_t)r; }

char* ShmComm::result_() { return result_base_; }

char* ShmComm::small_(int r, uint64_t e) {
  return small_base_ + kSmallBytes * (2 * (size_t)r + (size_t)(e & 1));
}

size_t ShmComm::small_bytes() const { return kSmallBytes; }

void ShmComm::backoff_(uint64_t& spins) {
  ++spins;
  if (spins < 4096) {
    CCMPI_RELAX();
  } else if (spins < 65536) {
    sched_yield();
  } else {
    struct timespec ts{0, 20000};
    nanosleep(&ts, nullptr);
  }
}

void ShmComm::timeout_(const char* what) {
  std::fprintf(stderr, "[ccmpi %s rank %d/%d] timeout after %.0fs in %s (deadlock or dead peer)\n",
               name_.c_str(), rank_, size_, timeout_s_, what);
  std::fflush(stderr);
  std::abort();
}

// ---------------------------------------------------------------------------
// point to point
// ---------------------------------------------------------------------------
namespace {

inline void ring_put(char* r, size_t cap, uint64_t pos, const char* src, size_t n) {
  size_t o = (size_t)(pos & (cap - 1));
  size_t a = std::min(n, cap - o);
  std::memcpy(r + o, src, a);
  if (n > a) std::memcpy(r, src + a, n - a);
}

inline void ring_get(const char* r, size_t cap, uint64_t pos, char* dst, size_t n) {
  size_t o = (size_t)(pos & (cap - 1));
  size_t a = std::min(n, cap - o);
  if (dst) {
    std::memcpy(dst, r + o, a);
    if (n > a) std::memcpy(dst + a, r, n - a);
  }
}

// ANY_TAG matches user tags only: the framework's own P2P schedules
// (p2p_algos.cpp) use negative internal tags that user receives never see.
inline bool tag_match(int want, int got) { return (want == ANY_TAG && got >= 0) || want == got; }

}  // namespace

bool ShmComm::progress_send_(int dest) {
  bool moved = false;
  auto& q = send_q_[dest];
  const size_t cap = ring_cap_;
  ChanCtl& c = *static_cast<ChanCtl*>(out_ctl_[dest]);
  char* rb = out_ring_[dest];
  uint64_t head = c.head.load(std::memory_order_relaxed);
  // the consumer's tail is re-read only when the cached value shows too little
  // room: a steady stream of small messages never pulls the consumer's line
  uint64_t& tail = peer_tail_[dest];
  while (!q.empty()) {
    RequestPtr r = q.front();
    size_t free_b = cap - (size_t)(head - tail);
    const size_t want = (r->header_sent ? 0 : kHdr) + (r->cap - r->done);
    if (free_b < want) {
      tail = c.tail.load(std::memory_order_acquire);
      free_b = cap - (size_t)(head - tail);
    }
    if (!r->header_sent) {
      if (free_b < kHdr) return moved;
      char hdr[kHdr];
      int32_t tag = r->tag, mg = 0x5a5a;
      uint64_t nb = r->cap;
      std::memcpy(hdr, &tag, 4);
      std::memcpy(hdr + 4, &mg, 4);
      std::memcpy(hdr + 8, &nb, 8);
      ring_put(rb, cap, head, hdr, kHdr);
      head += kHdr;
      free_b -= kHdr;
      r->header_sent = true;
      moved = true;
    }
    size_t n = std::min(free_b, r->cap - r->done);
    if (n > 0) {
      const char* src = r->owned.empty() ? r->buf : r->owned.data();
      ring_put(rb, cap, head, src + r->done, n);
      head += n;
      r->done += n;
      moved = true;
    }
    // one publication per (header + payload) that fits: the consumer sees the
    // whole message at once instead of the header first
    if (moved) c.head.store(head, std::memory_order_release);
    if (r->done == r->cap) {
      r->complete = true;
      q.pop_front();
      continue;
    }
    return moved;
  }
  return moved;
}

bool ShmComm::progress_recv_(int src) {
  bool moved = false;
  const size_t cap = ring_cap_;
  ChanCtl& c = *static_cast<ChanCtl*>(in_ctl_[src]);
  const char* rb = in_ring_[src];
  Cursor& cu = cur_[src];
  for (;;) {
    uint64_t head = c.head.load(std::memory_order_acquire);
    uint64_t tail = c.tail.load(std::memory_order_relaxed);
    size_t avail = (size_t)(head - tail);
    if (!cu.active) {
      if (avail < kHdr) return moved;
      char hdr[kHdr];
      ring_get(rb, cap, tail, hdr, kHdr);
      int32_t tag;
      uint64_t nb;
      std::memcpy(&tag, hdr, 4);
      std::memcpy(&nb, hdr + 8, 8);
      tail += kHdr;
      avail -= kHdr;
      c.tail.store(tail, std::memory_order_release);
      cu.active = true;
      cu.tag = tag;
      cu.nbytes = nb;
      cu.done = 0;
      cu.req.reset();
      cu.ux.reset();
      for (auto it = posted_.begin(); it != posted_.end(); ++it) {
        RequestPtr r = *it;
        if ((r->peer == ANY_SOURCE || r->peer == src) && tag_match(r->tag, tag)) {
          cu.req = r;
          posted_.erase(it);
          r->st_source = src;
          r->st_tag = tag;
          r->st_count = std::min<size_t>(nb, r->cap);
          r->truncated = nb > r->cap;
          break;
        }
      }
      if (!cu.req) {
        auto u = std::make_shared<Unexp>();
        u->tag = tag;
        u->data.resize(nb);
        u->complete = false;
        u->expect = nb;
        cu.ux = u;
        unexpected_[src].push_back(u);
      }
      moved = true;
    }
    size_t n = std::min(avail, cu.nbytes - cu.done);
    if (n > 0) {
      if (cu.req) {
        RequestPtr& r = cu.req;
        // copy the part that fits, drop the truncated remainder
        size_t fit = cu.done < r->cap ? std::min(n, r->cap - cu.done) : 0;
        if (fit) ring_get(rb, cap, tail, r->buf + cu.done, fit);
      } else {
        ring_get(rb, cap, tail, cu.ux->data.data() + cu.done, n);
      }
      tail += n;
      cu.done += n;
      c.tail.store(tail, std::memory_order_release);
      moved = true;
    }
    if (cu.done == cu.nbytes) {
      if (cu.req) {
        cu.req->done = cu.req->st_count;
        cu.req->complete = true;
      } else {
        cu.ux->complete = true;
      }
      cu.active = false;
      cu.req.reset();
      cu.ux.reset();
      continue;
    }
    return moved;
  }
}

bool ShmComm::progress() {
  bool moved = false;
  for (int d = 0; d < size_; ++d)
    if (!send_q_[d].empty()) moved |= progress_send_(d);
  for (int s = 0; s < size_; ++s) moved |= progress_recv_(s);
  // advance started non-blocking collectives (nbcoll.cpp): a rank waiting on
  // anything still forwards its collective rounds
  if (!nb_active_.empty()) nb_progress_();
  return moved;
}

bool ShmComm::try_match_unexpected_(const RequestPtr& r) {
  int lo = r->peer == ANY_SOURCE ? 0 : r->peer;
  int hi = r->peer == ANY_SOURCE ? size_ - 1 : r->peer;
  for (int s = lo; s <= hi; ++s) {
    auto& dq = unexpected_[s];
    for (auto it = dq.begin(); it != dq.end(); ++it) {
      auto u = *it;
      if (!tag_match(r->tag, u->tag)) continue;
      if (!u->complete) {
        // Finish streaming this message first so ordering is preserved.
        uint64_t spins = 0;
        double t0 = wtime();
        while (!u->complete) {
          if (!progress()) backoff_(spins);
          if ((spins & 1023) == 1023 && wtime() - t0 > timeout_s_) timeout_("recv (unexpected)");
        }
      }
      size_t nb = u->data.size();
      size_t fit = std::min(nb, r->cap);
      if (fit) std::memcpy(r->buf, u->data.data(), fit);
      r->st_source = s;
      r->st_tag = u->tag;
      r->st_count = fit;
      r->truncated = nb > r->cap;
      r->done = fit;
      r->complete = true;
      // iterator may be invalidated by progress(): re-find
      auto& dq2 = unexpected_[s];
      dq2.erase(std::find(dq2.begin(), dq2.end(), u));
      return true;
    }
  }
  return false;
}

void ShmComm::post_recv_(const RequestPtr& r) {
  if (r->peer == PROC_NULL) {
    r->complete = true;
    r->st_source = PROC_NULL;
    r->st_tag = ANY_TAG;
    return;
  }
  progress();
  if (try_match_unexpected_(r)) return;
  posted_.push_back(r);
}

RequestPtr ShmComm::isend(const void* buf, size_t nbytes, int dest, int tag) {
  if (tag < 0) throw std::invalid_argument("ccmpi: send tag must be >= 0");
  return isend_raw(buf, nbytes, dest, tag);
}

RequestPtr ShmComm::isend_raw(const void* buf, size_t nbytes, int dest, int tag) {
  if (g_p2p_trace_fine) p2p_trace_mark();
  auto r = std::make_shared<Request>();
  if (g_p2p_trace_fine) p2p_trace_mark();
  r->kind = Request::SEND;
  r->peer = dest;
  r->tag = tag;
  r->cap = nbytes;
  r->buf = const_cast<char*>(static_cast<const char*>(buf));
  if (dest == PROC_NULL) { r->complete = true; return r; }
  if (dest < 0 || dest >= size_) throw std::invalid_argument("ccmpi: invalid destination rank");
  send_q_[dest].push_back(r);
  if (g_p2p_trace_fine) p2p_trace_mark();
  progress_send_(dest);
  if (g_p2p_trace_fine) p2p_trace_mark();
  return r;
}

RequestPtr ShmComm::irecv(void* buf, size_t cap, int source, int tag) {
  if (source != ANY_SOURCE && source != PROC_NULL && (source < 0 || source >= size_))
    throw std::invalid_argument("ccmpi: invalid source rank");
  auto r = std::make_shared<Request>();
  r->kind = Request::RECV;
  r->peer = source;
  r->tag = tag;
  r->buf = static_cast<char*>(buf);
  r->cap = cap;
  post_recv_(r);
  return r;
}

void ShmComm::wait(const RequestPtr& r) {
  uint64_t spins = 0;
  double t0 = wtime();
  while (!r->complete) {
    if (!progress()) backoff_(spins);
    else spins = 0;
    if ((++spins & 1023) == 0 && wtime() - t0 > timeout_s_) timeout_(r->kind == Request::SEND ? "send" : "recv");
  }
  if (r->truncated)
    throw std::runtime_error("ccmpi: message truncated (receive buffer too small)");
}

bool ShmComm::test(const RequestPtr& r) {
  if (!r->complete) progress();
  return r->complete;
}

void ShmComm::waitall(const std::vector<RequestPtr>& rs) {
  for (auto& r : rs) wait(r);
}

int ShmComm::waitany(const std::vector<RequestPtr>& rs) {
  if (rs.empty()) return -1;
  uint64_t spins = 0;
  double t0 = wtime();
  for (;;) {
    for (size_t i = 0; i < rs.size(); ++i)
      if (rs[i] && rs[i]->complete) return (int)i;
    if (!progress()) backoff_(spins);
    if ((++spins & 1023) == 0 && wtime() - t0 > timeout_s_) timeout_("waitany");
  }
}

void ShmComm::send(const void* buf, size_t nbytes, int dest, int tag) {
  wait(isend(buf, nbytes, dest, tag));
}

RequestPtr ShmComm::recv(void* buf, size_t cap, int source, int tag) {
  auto r = irecv(buf, cap, source, tag);
  wait(r);
  return r;
}

RequestPtr ShmComm::sendrecv(const void* sbuf, size_t sbytes, int dest, int stag, void* rbuf,
                             size_t rcap, int source, int rtag) {
  auto rr = irecv(rbuf, rcap, source, rtag);
  auto sr = isend(sbuf, sbytes, dest, stag);
  wait(sr);
  wait(rr);
  return rr;
}

bool ShmComm::iprobe(int source, int tag, int* src_out, int* tag_out, size_t* bytes_out) {
  progress();
  int lo = source == ANY_SOURCE ? 0 : source;
  int hi = source == ANY_SOURCE ? size_ - 1 : source;
  for (int s = lo; s <= hi; ++s) {
    for (auto& u : unexpected_[s]) {
      if (tag_match(tag, u->tag)) {
        *src_out = s;
        *tag_out = u->tag;
        *bytes_out = u->expect;
        return true;
      }
    }
  }
  return false;
}

void ShmComm::probe(int source, int tag, int* src_out, int* tag_out, size_t* bytes_out) {
  uint64_t spins = 0;
  double t0 = wtime();
  while (!iprobe(source, tag, src_out, tag_out, bytes_out)) {
    backoff_(spins);
    if ((spins & 1023) == 0 && wtime() - t0 > timeout_s_) timeout_("probe");
  }
}

// ---------------------------------------------------------------------------
// collectives
// ---------------------------------------------------------------------------
// Flat epoch barrier: every rank stores its own flag (no shared counter, no
// contended line) and waits until every other rank's flag reaches the epoch.
void ShmComm::sync_epoch_(uint64_t e) {
  flag_[rank_]->store(e, std::memory_order_release);
  for (int j = 0; j < size_; ++j) {
    if (j == rank_ || flag_[j]->load(std::memory_order_acquire) >= e) continue;
    uint64_t spins = 0;
    double t0 = wtime();
    while (flag_[j]->load(std::memory_order_acquire) < e) {
      // keep point-to-point traffic moving while we wait (MPI-style progress)
      bool moved = false;
      if (!posted_.empty() || (spins & 63) == 0) moved = progress();
      if (!moved) backoff_(spins);
      if ((spins & 1023) == 1023 && wtime() - t0 > timeout_s_) timeout_("barrier");
    }
  }
}

void ShmComm::slot_barrier_() { sync_epoch_(++bar_epoch_); }

void ShmComm::barrier() {
  if (size_ == 1) return;
  slot_barrier_();
}

void ShmComm::bcast(void* buf, size_t nbytes, int root) {
  if (size_ == 1 || nbytes == 0) return;
  char* b = static_cast<char*>(buf);
  if (nbytes <= kSmallBytes) {
    const uint64_t e = ++bar_epoch_;
    if (rank_ == root) std::memcpy(small_(root, e), b, nbytes);
    sync_epoch_(e);
    if (rank_ != root) std::memcpy(b, small_(root, e), nbytes);
    return;
  }
  // staged through the root's slot, not `result`: slots are only read between the
  // two barriers of a collective, while a rooted collective's root may still be
  // copying `result` out after the previous call's last barrier (Reduce, then a
  // Bcast from another root, overwrote the Reduce result under load)
  const size_t S = slot_bytes();
  for (size_t off = 0; off < nbytes; off += S) {
    size_t c = std::min(S, nbytes - off);
    if (rank_ == root) std::memcpy(slot_(root), b + off, c);
    slot_barrier_();
    if (rank_ != root) std::memcpy(b + off, slot_(root), c);
    slot_barrier_();
  }
}

void ShmComm::allreduce(const void* sbuf, void* rbuf, size_t count, int dt, int op) {
  const size_t es = dtype_size(dt);
  if (!reduce_supported(dt, op)) reduce_inplace(nullptr, nullptr, 0, dt, op);  // throws
  const char* src = sbuf ? static_cast<const char*>(sbuf) : static_cast<const char*>(rbuf);
  char* dst = static_cast<char*>(rbuf);
  if (size_ == 1) {
    if (src != dst) std::memmove(dst, src, count * es);
    return;
  }
  if (count * es <= small_allreduce_max_) {
    // one sync: publish, then every rank reduces all p inputs itself in rank
    // order (bitwise identical everywhere); epoch-parity double buffering makes
    // the next call safe without a trailing barrier
    const uint64_t e = ++bar_epoch_;
    std::memcpy(small_(rank_, e), src, count * es);
    sync_epoch_(e);
    if (dst != small_(0, e)) std::memcpy(dst, small_(0, e), count * es);
    for (int j = 1; j < size_; ++j) reduce_inplace(dst, small_(j, e), count, dt, op);
    return;
  }
  const size_t per = slot_bytes() / es;
  for (size_t off = 0; off < count; off += per) {
    const size_t n = std::min(per, count - off);
    std::memcpy(slot_(rank_), src + off * es, n * es);
    slot_barrier_();
    const size_t lo = n * rank_ / size_, hi = n * (rank_ + 1) / size_;
    if (hi > lo) {
      char* res = result_() + lo * es;
      std::memcpy(res, slot_(0) + lo * es, (hi - lo) * es);
      for (int j = 1; j < size_; ++j) reduce_inplace(res, slot_(j) + lo * es, hi - lo, dt, op);
    }
    slot_barrier_();
    std::memcpy(dst + off * es, result_(), n * es);
  }
}

void ShmComm::reduce(const void* sbuf, void* rbuf, size_t count, int dt, int op, int root) {
  const size_t es = dtype_size(dt);
  if (!reduce_supported(dt, op)) reduce_inplace(nullptr, nullptr, 0, dt, op);
  const char* src = sbuf ? static_cast<const char*>(sbuf) : static_cast<const char*>(rbuf);
  char* dst = static_cast<char*>(rbuf);
  if (size_ == 1) {
    if (src != dst) std::memmove(dst, src, count * es);
    return;
  }
  const size_t per = slot_bytes() / es;
  for (size_t off = 0; off < count; off += per) {
    const size_t n = std::min(per, count - off);
    std::memcpy(slot_(rank_), src + off * es, n * es);
    slot_barrier_();
    const size_t lo = n * rank_ / size_, hi = n * (rank_ + 1) / size_;
    if (hi > lo) {
      char* res = result_() + lo * es;
      std::memcpy(res, slot_(0) + lo * es, (hi - lo) * es);
      for (int j = 1; j < size_; ++j) reduce_inplace(res, slot_(j) + lo * es, hi - lo, dt, op);
    }
    slot_barrier_();
    if (rank_ == root) std::memcpy(dst + off * es, result_(), n * es);
  }
  // the root's copy-out must finish before the next collective reuses `result`;
  // every collective writes `result` only after its first barrier, so no extra sync.
}

void ShmComm::reduce_scatter(const void* sbuf, void* rbuf, const std::vector<size_t>& counts,
                             int dt, int op) {
  if ((int)counts.size() != size_) throw std::invalid_argument("ccmpi: counts must have one entry per rank");
  const size_t es = dtype_size(dt);
  if (!reduce_supported(dt, op)) reduce_inplace(nullptr, nullptr, 0, dt, op);
  std::vector<size_t> displ(size_, 0);
  size_t maxc = 0;
  for (int i = 1; i < size_; ++i) displ[i] = displ[i - 1] + counts[i - 1];
  for (auto c : counts) maxc = std::max(maxc, c);
  const char* src = sbuf ? static_cast<const char*>(sbuf) : static_cast<const char*>(rbuf);
  char* dst = static_cast<char*>(rbuf);
  if (size_ == 1) {
    if (src != dst) std::memmove(dst, src, counts[0] * es);
    return;
  }
  // in-place: the result overwrites the head of rbuf, which aliases input
  // blocks that later rounds still read: work from a private copy then.
  const size_t per = slot_bytes() / (es * size_);
  if (per == 0) throw std::runtime_error("ccmpi: slot too small for reduce_scatter");
  std::vector<char> inplace_copy;
  if (src == dst && maxc > per) {
    size_t total = displ[size_ - 1] + counts[size_ - 1];
    inplace_copy.assign(src, src + total * es);
    src = inplace_copy.data();
  }
  for (size_t off = 0; off < maxc; off += per) {
    char* mine = slot_(rank_);
    for (int b = 0; b < size_; ++b) {
      if (counts[b] > off) {
        size_t nb = std::min(per, counts[b] - off);
        std::memcpy(mine + (size_t)b * per * es, src + (displ[b] + off) * es, nb * es);
      }
    }
    slot_barrier_();
    if (counts[rank_] > off) {
      size_t n = std::min(per, counts[rank_] - off);
      char* out = dst + off * es;
      const size_t boff = (size_t)rank_ * per * es;
      std::memcpy(out, slot_(0) + boff, n * es);
      for (int j = 1; j < size_; ++j) reduce_inplace(out, slot_(j) + boff, n, dt, op);
    }
    slot_barrier_();
  }
}

void ShmComm::reduce_scatter_block(const void* sbuf, void* rbuf, size_t count, int dt, int op) {
  std::vector<size_t> counts(size_, count);
  reduce_scatter(sbuf, rbuf, counts, dt, op);
}

void ShmComm::allgatherv(const void* sbuf, size_t nbytes, void* rbuf,
                         const std::vector<size_t>& counts, const std::vector<size_t>& displs) {
  if ((int)counts.size() != size_ || (int)displs.size() != size_)
    throw std::invalid_argument("ccmpi: counts/displs must have one entry per rank");
  char* dst = static_cast<char*>(rbuf);
  const char* src = sbuf ? static_cast<const char*>(sbuf) : dst + displs[rank_];
  if (size_ == 1) {
    if (dst + displs[0] != src) std::memmove(dst + displs[0], src, nbytes);
    return;
  }
  size_t maxc = 0;
  for (auto c : counts) maxc = std::max(maxc, c);
  const size_t S = slot_bytes();
  for (size_t off = 0; off < maxc; off += S) {
    if (nbytes > off) std::memcpy(slot_(rank_), src + off, std::min(S, nbytes - off));
    slot_barrier_();
    for (int j = 0; j < size_; ++j) {
      if (counts[j] > off) {
        size_t c = std::min(S, counts[j] - off);
        if (!(j == rank_ && sbuf == nullptr)) std::memcpy(dst + displs[j] + off, slot_(j), c);
      }
    }
    slot_barrier_();
  }
}

void ShmComm::allgather(const void* sbuf, size_t nbytes, void* rbuf) {
  if (size_ > 1 && nbytes <= kSmallBytes) {
    char* dst = static_cast<char*>(rbuf);
    const char* src = sbuf ? static_cast<const char*>(sbuf) : dst + nbytes * (size_t)rank_;
    const uint64_t e = ++bar_epoch_;
    std::memcpy(small_(rank_, e), src, nbytes);
    sync_epoch_(e);
    for (int j = 0; j < size_; ++j)
      if (dst + nbytes * (size_t)j != small_(j, e)) std::memcpy(dst + nbytes * (size_t)j, small_(j, e), nbytes);
    return;
  }
  std::vector<size_t> counts(size_, nbytes), displs(size_);
  for (int i = 0; i < size_; ++i) displs[i] = nbytes * (size_t)i;
  allgatherv(sbuf, nbytes, rbuf, counts, displs);
}

void ShmComm::gatherv(const void* sbuf, size_t nbytes, void* rbuf, const std::vector<size_t>& counts,
                      const std::vector<size_t>& displs, int root) {
  char* dst = static_cast<char*>(rbuf);
  const char* src = static_cast<const char*>(sbuf);
  if (size_ == 1) {
    if (src && dst + displs[0] != src) std::memmove(dst + displs[0], src, nbytes);
    return;
  }
  // counts are significant only at root: agree on the round count first
  uint64_t mine = nbytes, maxc = 0;
  allreduce(&mine, &maxc, 1, DT_U64, OP_MAX);
  const size_t S = slot_bytes();
  for (size_t off = 0; off < maxc; off += S) {
    if (nbytes > off && src) std::memcpy(slot_(rank_), src + off, std::min(S, nbytes - off));
    slot_barrier_();
    if (rank_ == root) {
      for (int j = 0; j < size_; ++j) {
        if (counts[j] > off) {
          if (j == rank_ && !src) continue;
          std::memcpy(dst + displs[j] + off, slot_(j), std::min(S, counts[j] - off));
        }
      }
    }
    slot_barrier_();
  }
}

void ShmComm::gather(const void* sbuf, size_t nbytes, void* rbuf, int root) {
  std::vector<size_t> counts(size_, nbytes), displs(size_);
  for (int i = 0; i < size_; ++i) displs[i] = nbytes * (size_t)i;
  gatherv(sbuf, nbytes, rbuf, counts, displs, root);
}

void ShmComm::scatterv(const void* sbuf, const std::vector<size_t>& counts,
                       const std::vector<size_t>& displs, void* rbuf, size_t nbytes, int root) {
  const char* src = static_cast<const char*>(sbuf);
  char* dst = static_cast<char*>(rbuf);
  if (size_ == 1) {
    if (dst && src + displs[0] != dst) std::memmove(dst, src + displs[0], nbytes);
    return;
  }
  uint64_t mine = nbytes, maxc = 0;
  allreduce(&mine, &maxc, 1, DT_U64, OP_MAX);
  const size_t S = slot_bytes();
  for (size_t off = 0; off < maxc; off += S) {
    if (rank_ == root) {
      for (int j = 0; j < size_; ++j)
        if (counts[j] > off) std::memcpy(slot_(j), src + displs[j] + off, std::min(S, counts[j] - off));
    }
    slot_barrier_();
    if (nbytes > off && dst && !(rank_ == root && dst == src + displs[root]))
      std::memcpy(dst + off, slot_(rank_), std::min(S, nbytes - off));
    slot_barrier_();
  }
}

void ShmComm::scatter(const void* sbuf, size_t nbytes, void* rbuf, int root) {
  std::vector<size_t> counts(size_, nbytes), displs(size_);
  for (int i = 0; i < size_; ++i) displs[i] = nbytes * (size_t)i;
  scatterv(sbuf, counts, displs, rbuf, nbytes, root);
}

void ShmComm::alltoallv(const void* sbuf, const std::vector<size_t>& scounts,
                        const std::vector<size_t>& sdispls, void* rbuf,
                        const std::vector<size_t>& rcounts, const std::vector<size_t>& rdispls) {
  const char* src = static_cast<const char*>(sbuf);
  char* dst = static_cast<char*>(rbuf);
  if (size_ == 1) {
    if (src + sdispls[0] != dst + rdispls[0]) std::memmove(dst + rdispls[0], src + sdispls[0], scounts[0]);
    return;
  }
  uint64_t mine = 0, maxc = 0;
  for (auto c : scounts) mine = std::max<uint64_t>(mine, c);
  allreduce(&mine, &maxc, 1, DT_U64, OP_MAX);
  const size_t cs = (slot_bytes() / size_) / 64 * 64;
  for (size_t off = 0; off < maxc; off += cs) {
    char* mine_slot = slot_(rank_);
    for (int b = 0; b < size_; ++b)
      if (scounts[b] > off) std::memcpy(mine_slot + (size_t)b * cs, src + sdispls[b] + off, std::min(cs, scounts[b] - off));
    slot_barrier_();
    for (int j = 0; j < size_; ++j)
      if (rcounts[j] > off) std::memcpy(dst + rdispls[j] + off, slot_(j) + (size_t)rank_ * cs, std::min(cs, rcounts[j] - off));
    slot_barrier_();
  }
}

void ShmComm::alltoall(const void* sbuf, size_t block_bytes, void* rbuf) {
  const char* src = static_cast<const char*>(sbuf);
  char* dst = static_cast<char*>(rbuf);
  if (size_ == 1) {
    if (src && src != dst) std::memmove(dst, src, block_bytes);
    return;
  }
  if (!src) src = dst;  // in place: inputs go to the slots before anyone writes
  if (block_bytes * (size_t)size_ <= kSmallBytes) {
    const uint64_t e = ++bar_epoch_;
    std::memcpy(small_(rank_, e), src, block_bytes * (size_t)size_);
    sync_epoch_(e);
    for (int j = 0; j < size_; ++j)
      std::memcpy(dst + (size_t)j * block_bytes, small_(j, e) + (size_t)rank_ * block_bytes, block_bytes);
    return;
  }
  const size_t cs = (slot_bytes() / size_) / 64 * 64;
  for (size_t off = 0; off < block_bytes; off += cs) {
    const size_t c = std::min(cs, block_bytes - off);
    char* mine_slot = slot_(rank_);
    for (int b = 0; b < size_; ++b) std::memcpy(mine_slot + (size_t)b * cs, src + (size_t)b * block_bytes + off, c);
    slot_barrier_();
    for (int j = 0; j < size_; ++j)
      std::memcpy(dst + (size_t)j * block_bytes + off, slot_(j) + (size_t)rank_ * cs, c);
    slot_barrier_();
  }
}

void ShmComm::scan(const void* sbuf, void* rbuf, size_t count, int dt, int op, bool exclusive) {
  const size_t es = dtype_size(dt);
  if (!reduce_supported(dt, op)) reduce_inplace(nullptr, nullptr, 0, dt, op);
  const char* src = sbuf ? static_cast<const char*>(sbuf) : static_cast<const char*>(rbuf);
  char* dst = static_cast<char*>(rbuf);
  const size_t per = slot_bytes() / es;
  for (size_t off = 0; off < count; off += per) {
    const size_t n = std::min(per, count - off);
    std::memcpy(slot_(rank_), src + off * es, n * es);
    slot_barrier_();
    const int upto = exclusive ? rank_ - 1 : rank_;
    if (upto >= 0) {
      char* out = dst + off * es;
      std::memcpy(out, slot_(0), n * es);
      for (int j = 1; j <= upto; ++j) reduce_inplace(out, slot_(j), n, dt, op);
    }
    slot_barrier_();
  }
}

std::shared_ptr<ShmComm> ShmComm::split(int color, int key) {
  struct Ent { int32_t color, key, rank; };
  Ent me{color, key, rank_};
  std::vector<Ent> all(size_);
  allgather(&me, sizeof(Ent), all.data());
  const uint64_t seq = split_seq_++;
  if (color < 0) return nullptr;
  std::vector<Ent> mem;
  for (auto& e : all)
    if (e.color == color) mem.push_back(e);
  std::stable_sort(mem.begin(), mem.end(), [](const Ent& a, const Ent& b) {
    return a.key != b.key ? a.key < b.key : a.rank < b.rank;
  });
  int nr = -1;
  for (size_t i = 0; i < mem.size(); ++i)
    if (mem[i].rank == rank_) nr = (int)i;
  std::string child = "ccmpi_" + hex64(fnv1a(name_ + "|" + std::to_string(seq) + "|" + std::to_string(color)));
  auto c = std::make_shared<ShmComm>(child, nr, (int)mem.size());
  for (size_t i = 0; i < mem.size(); ++i) c->world_ranks_[i] = world_ranks_[mem[i].rank];
  c->timeout_s_ = timeout_s_;
  return c;
}

}  // namespace ccmpi
