// Host plane of the framework: an intra-node, shared-memory message-passing
// runtime that replaces what the reference delegates to mpi4py + libmpi
// (reference: mpi_wrapper/comm.py:1-199 calls Comm.{Send,Recv,Isend,Irecv,
// Sendrecv,Allreduce,Allgather,Reduce_scatter_block,Alltoall,Split,Barrier}).
//
// Design (not a port of any MPI implementation):
//   * one POSIX shm segment per communicator, created collectively, unlinked as
//     soon as every member has mapped it (nothing leaks in /dev/shm);
//   * point-to-point = one single-producer/single-consumer byte ring per ordered
//     rank pair carrying {tag, nbytes} framed messages; a per-process progress
//     engine drives every outstanding Isend/Irecv (so Waitall over a full
//     all-to-all never deadlocks) and keeps an unexpected-message queue for
//     tag/source matching;
//   * collectives do NOT go through the P2P rings: they use a per-rank slot
//     region + a shared result region + a monotonic-counter barrier, so every
//     rank reduces a disjoint 1/p of each chunk in rank order 0..p-1
//     (deterministic, bitwise identical results on all ranks).
//   * this plane also bootstraps the device plane (IPC handle / RCCL id
//     exchange) — see csrc/device/device_comm.hip.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <memory>
#include <string>
#include <vector>

namespace ccmpi {

enum DType : int {
  DT_I8 = 0, DT_U8, DT_I16, DT_U16, DT_I32, DT_U32, DT_I64, DT_U64,
  DT_F16, DT_BF16, DT_F32, DT_F64, DT_BOOL, DT_C64, DT_C128, DT_BYTE,
  DT_COUNT
};

enum ROp : int {
  OP_SUM = 0, OP_PROD, OP_MIN, OP_MAX, OP_LAND, OP_LOR, OP_LXOR,
  OP_BAND, OP_BOR, OP_BXOR, OP_REPLACE, OP_COUNT
};

constexpr int ANY_SOURCE = -1;
constexpr int ANY_TAG = -1;
constexpr int PROC_NULL = -2;

size_t dtype_size(int dt);
// dst[i] = dst[i] (op) src[i] for n elements. Throws for unsupported combos.
void reduce_inplace(void* dst, const void* src, size_t n, int dt, int op);
bool reduce_supported(int dt, int op);

struct Segment;  // opaque shm layout
class ShmComm;

// A started non-blocking collective: a schedule of P2P rounds (nbcoll.cpp).
class NbColl {
 public:
  virtual ~NbColl() = default;
  // Post round k's messages; false when the schedule has no round k.
  virtual bool post(ShmComm& c, int k) = 0;
  // Local work once round k's messages completed.
  virtual void finish(int /*k*/) {}

  std::vector<std::shared_ptr<struct Request>> reqs;
  int round = -1;
  bool done = false;
  std::string err;
  int tag = 0;  // internal tag base; round k uses tag - k
  std::vector<char> tmp;

 protected:
  void recv(ShmComm& c, void* b, size_t n, int src, int k);
  void send(ShmComm& c, const void* b, size_t n, int dst, int k);
};
using NbCollPtr = std::shared_ptr<NbColl>;

struct Request {
  enum Kind { SEND, RECV } kind;
  int peer = 0;
  int tag = 0;
  char* buf = nullptr;       // recv destination / send source
  size_t cap = 0;            // recv capacity or send size
  size_t done = 0;           // bytes moved so far
  bool header_sent = false;  // send side
  bool complete = false;
  bool truncated = false;
  int st_source = -1, st_tag = -1;
  size_t st_count = 0;       // bytes actually received
  std::vector<char> owned;   // send: private copy for small eager sends
};
using RequestPtr = std::shared_ptr<Request>;

class ShmComm : public std::enable_shared_from_this<ShmComm> {
 public:
  // Create (collectively) a communicator of `size` ranks over segment `name`.
  ShmComm(const std::string& name, int rank, int size);
  ~ShmComm();
  ShmComm(const ShmComm&) = delete;
  ShmComm& operator=(const ShmComm&) = delete;

  // Bootstraps the world communicator from the launcher environment
  // (CCMPI_* from our launcher, PMI_* from Hydra mpiexec, OMPI_* from Open MPI,
  // RANK/WORLD_SIZE from torchrun).  Singleton if none is set.
  static std::shared_ptr<ShmComm> world();

  int rank() const { return rank_; }
  int size() const { return size_; }
  const std::string& name() const { return name_; }
  int world_rank_of(int r) const { return world_ranks_[r]; }
  const std::vector<int>& world_ranks() const { return world_ranks_; }

  // ---- point to point -------------------------------------------------
  RequestPtr isend(const void* buf, size_t nbytes, int dest, int tag);
  RequestPtr irecv(void* buf, size_t cap, int source, int tag);
  void wait(const RequestPtr& r);
  bool test(const RequestPtr& r);
  void waitall(const std::vector<RequestPtr>& rs);
  int waitany(const std::vector<RequestPtr>& rs);
  void send(const void* buf, size_t nbytes, int dest, int tag);
  // returns request holding status
  RequestPtr recv(void* buf, size_t cap, int source, int tag);
  RequestPtr sendrecv(const void* sbuf, size_t sbytes, int dest, int stag,
                      void* rbuf, size_t rcap, int source, int rtag);
  // Probe: blocks until a matching message is available; returns (src, tag, bytes).
  void probe(int source, int tag, int* src_out, int* tag_out, size_t* bytes_out);
  bool iprobe(int source, int tag, int* src_out, int* tag_out, size_t* bytes_out);

  // ---- the reference's hand-written collectives as native P2P schedules --
  // (p2p_algos.cpp; same message pattern as mpi_wrapper/comm.py, internal tags)
  // myAllreduce (comm.py:63-107): reduce to rank 0 in rank order, then send back.
  void my_reduce_bcast(const void* src, void* dst, size_t count, int dt, int op);
  // myAlltoall (comm.py:110-159): every irecv posted before any isend, waitall.
  void my_alltoall_nb(const void* src, void* dst, size_t block_bytes);
  // myAlltoall2 (comm.py:162-199): pairwise sendrecv in rank order.
  void my_alltoall_pairwise(const void* src, void* dst, size_t block_bytes);
  // ring reduce-scatter + all-gather, and recursive halving/doubling.
  void my_ring_allreduce(const void* src, void* dst, size_t count, int dt, int op);
  void my_rhd_allreduce(const void* src, void* dst, size_t count, int dt, int op);

  // ---- collectives (all ranks, same order) ----------------------------
  void barrier();
  void bcast(void* buf, size_t nbytes, int root);
  void allreduce(const void* sbuf, void* rbuf, size_t count, int dt, int op);
  void reduce(const void* sbuf, void* rbuf, size_t count, int dt, int op, int root);
  void reduce_scatter_block(const void* sbuf, void* rbuf, size_t count, int dt, int op);
  void reduce_scatter(const void* sbuf, void* rbuf, const std::vector<size_t>& counts,
                      int dt, int op);
  void allgather(const void* sbuf, size_t nbytes, void* rbuf);
  void allgatherv(const void* sbuf, size_t nbytes, void* rbuf,
                  const std::vector<size_t>& counts, const std::vector<size_t>& displs);
  void gather(const void* sbuf, size_t nbytes, void* rbuf, int root);
  void gatherv(const void* sbuf, size_t nbytes, void* rbuf, const std::vector<size_t>& counts,
               const std::vector<size_t>& displs, int root);
  void scatter(const void* sbuf, size_t nbytes, void* rbuf, int root);
  void scatterv(const void* sbuf, const std::vector<size_t>& counts,
                const std::vector<size_t>& displs, void* rbuf, size_t nbytes, int root);
  void alltoall(const void* sbuf, size_t block_bytes, void* rbuf);
  void alltoallv(const void* sbuf, const std::vector<size_t>& scounts,
                 const std::vector<size_t>& sdispls, void* rbuf,
                 const std::vector<size_t>& rcounts, const std::vector<size_t>& rdispls);
  void scan(const void* sbuf, void* rbuf, size_t count, int dt, int op, bool exclusive);

  // ---- non-blocking collectives (nbcoll.cpp): schedules of P2P rounds on
  // internal tags, advanced by every progress() call until complete
  NbCollPtr ibarrier();
  NbCollPtr ibcast(void* buf, size_t nbytes, int root);
  NbCollPtr iallreduce(const void* sbuf, void* rbuf, size_t count, int dt, int op);
  NbCollPtr iallgather(const void* sbuf, size_t nbytes, void* rbuf);
  NbCollPtr ialltoall(const void* sbuf, size_t block_bytes, void* rbuf);
  // sbuf == nullptr: in place, rbuf holds the p*count input and receives block rank()
  NbCollPtr ireduce_scatter_block(const void* sbuf, void* rbuf, size_t count, int dt, int op);
  bool nb_test(const NbCollPtr& c);
  void nb_wait(const NbCollPtr& c);
  size_t nb_active() const { return nb_active_.size(); }
  RequestPtr isend_internal(const void* buf, size_t nbytes, int dest, int tag);  // tag < 0

  // Collective: split by (color, key).  Returns nullptr for color < 0 (UNDEFINED).
  std::shared_ptr<ShmComm> split(int color, int key);
  std::shared_ptr<ShmComm> dup() { return split(0, rank_); }

  size_t slot_bytes() const;
  size_t small_bytes() const;
  size_t ring_bytes() const;

  // Progress every outstanding request once; returns true if anything moved.
  bool progress();

 private:
  RequestPtr isend_raw(const void* buf, size_t nbytes, int dest, int tag);  // no user-tag check
  void attach_();
  void sync_epoch_(uint64_t e);
  void slot_barrier_();
  char* small_(int r, uint64_t e);
  char* slot_(int r);
  char* result_();
  bool try_match_unexpected_(const RequestPtr& r);
  void post_recv_(const RequestPtr& r);
  bool progress_send_(int dest);
  bool progress_recv_(int src);
  void backoff_(uint64_t& spins);
  [[noreturn]] void timeout_(const char* what);
  NbCollPtr nb_start_(NbCollPtr c);
  bool nb_advance_(NbColl& c);
  void nb_progress_();

  std::string name_;
  int rank_, size_;
  std::vector<int> world_ranks_;
  Segment* seg_ = nullptr;
  size_t seg_bytes_ = 0;
  uint64_t bar_epoch_ = 0;
  uint64_t split_seq_ = 0;
  double timeout_s_ = 600.0;

  // progress engine state
  std::vector<std::deque<RequestPtr>> send_q_;   // per dest, FIFO
  std::deque<RequestPtr> posted_;                 // posted recvs, posting order
  struct Unexp { int tag; std::vector<char> data; bool complete; size_t expect; };
  std::vector<std::deque<std::shared_ptr<Unexp>>> unexpected_;  // per source
  // per-source receive cursor (the message currently streaming off the ring)
  struct Cursor { bool active = false; int tag = 0; size_t nbytes = 0; size_t done = 0;
                  RequestPtr req; std::shared_ptr<Unexp> ux; };
  std::vector<Cursor> cur_;
  // this rank's channel control blocks (opaque ChanCtl*) and rings, by peer
  std::vector<void*> out_ctl_, in_ctl_;
  std::vector<char*> out_ring_, in_ring_;
  size_t ring_cap_ = 0;
  std::vector<std::atomic<uint64_t>*> flag_;  // per-rank epoch flags
  char* small_base_ = nullptr;
  size_t small_allreduce_max_ = 1024;  // single-sync all-reduce up to this many bytes (measured crossover)
  char* slot_base_ = nullptr;
  char* result_base_ = nullptr;
  std::vector<uint64_t> peer_tail_;  // last tail read from each out-channel's consumer

  // started non-blocking collectives (held until complete), tag sequence
  std::vector<NbCollPtr> nb_active_;
  uint64_t nb_seq_ = 0;
  bool nb_in_progress_ = false;
};

double wtime();
std::string job_id_from_env();
extern bool g_p2p_trace_on;              // p2p_algos.cpp: CCMPI_P2P_TRACE
extern bool g_p2p_trace_fine;            // CCMPI_P2P_TRACE=2: marks inside isend_raw
void p2p_trace_mark();                   // one timestamp (when tracing is on)
std::vector<double> p2p_trace_take();   // reduce->bcast phase timestamps since the last take

}  // namespace ccmpi
