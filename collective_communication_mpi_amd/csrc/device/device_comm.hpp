// Device communicator: one per (host communicator, process).  Owns
//  * the uncached signal buffer peers write flags into (IPC-exported),
//  * per-CTA epoch counters,
//  * the device-resident PeerTable (peer signal buffers + symmetric segments),
//  * a symmetric scratch segment used to stage non-registered tensors,
//  * optionally an RCCL communicator (library baseline + P2P schedules).
// Bootstrap data (IPC handles, RCCL unique id) is exchanged by the Python
// layer over the host plane; this class never talks to other processes itself.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "collectives.hpp"
#include "common.hpp"
#include "gemm_common.hpp"

namespace ccmpi {
namespace dev {

struct SegInfo {
  char* local = nullptr;   // this rank's base
  uint64_t bytes = 0;
  bool owned = false;      // allocated by us (freed in dtor)
  bool dynamic = false;    // on-demand registration slot (searched only by calls that registered)
};

class DeviceComm {
 public:
  DeviceComm(int rank, int size, int device, uint64_t scratch_bytes);
  ~DeviceComm();

  int rank() const { return rank_; }
  int size() const { return size_; }
  int device() const { return device_; }

  // ---- bootstrap ---------------------------------------------------------
  std::string signal_handle() const;                       // IPC handle bytes of my Signals
  void connect(const std::vector<std::string>& sig_handles);
  // Register a local range as symmetric segment `seg` (collective, same index
  // on every rank).  Returns (handle bytes, offset from allocation base).
  std::pair<std::string, uint64_t> export_range(uint64_t ptr) const;
  int add_segment(uint64_t local_ptr, uint64_t bytes,
                  const std::vector<std::string>& handles, const std::vector<uint64_t>& offsets);
  // on-demand registration slot (see device_comm.cpp); returns the slot index
  int set_segment(int s, uint64_t local_ptr, uint64_t bytes, const std::vector<std::string>& handles,
                  const std::vector<uint64_t>& offsets, const std::vector<std::string>& keys);
  void clear_segment(int s);
  int num_segments() const { return (int)segs_.size(); }
  int scratch_segment() const { return 0; }
  uint64_t scratch_bytes() const { return segs_.empty() ? 0 : segs_[0].bytes; }
  uint64_t scratch_ptr() const { return segs_.empty() ? 0 : (uint64_t)segs_[0].local; }
  // (segment, offset) of a local pointer, or -1 if not inside a segment; on-demand
  // slots count only with `dynamic` (a call whose tensors were registered for it)
  int find(uint64_t ptr, uint64_t nbytes, uint64_t* off, bool dynamic = false) const;

  // ---- hand-written collectives (stream-ordered, graph-capturable) ----------
  // `symmetric`: caller guarantees every rank passes registered buffers, so
  // no staging/chunking is needed.  Otherwise inputs are staged through the
  // scratch segment in chunks whose size is identical on all ranks.
  void allreduce(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, int algo,
                 uint64_t stream, int max_blocks, bool symmetric);
  // Two-shot all-reduce whose reduce-scatter lands in the (registered, symmetric)
  // source itself -- rank r's reduced shard r overwrites its own source shard r,
  // which no peer reads -- and whose all-gather pulls the shards into `out`, a
  // LOCAL buffer that needs no registration.  The source is clobbered: it is the
  // scratch of a GEMM's partial product (TP row-parallel output, dX partial).
  void allreduce_to_local(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, uint64_t stream,
                          int max_blocks);
  void reduce_scatter(uint64_t in, uint64_t out, uint64_t count_per_rank, int dtype, int op,
                      uint64_t stream, int max_blocks, bool symmetric);
  // mode: A2A_PULL (default) or A2A_PUSH (every rank's output registered: the
  // input is written into every peer's output block `me`; the input stays local)
  void allgather(uint64_t in, uint64_t out, uint64_t bytes_per_rank, uint64_t stream, int max_blocks,
                 bool symmetric, int mode = 0);
  // mode: A2A_PULL (default; staged for in-place / unregistered input) or A2A_PUSH
  // (symmetric only: every rank's output registered, peer writes into it)
  // Ragged all-to-all (push into every rank's registered output): per-peer byte
  // offsets / lengths, all multiples of 16; grid_bytes = the largest total send of
  // any rank (the grid must match across ranks).
  void alltoallv(uint64_t in, uint64_t out, uint64_t out_bytes, const std::vector<uint64_t>& soff,
                 const std::vector<uint64_t>& doff, const std::vector<uint64_t>& len, uint64_t grid_bytes,
                 uint64_t stream, int max_blocks);
  // Ragged all-to-all with device-resident counts: `counts` (p int64, this rank's
  // send counts) and the output capacity are staged into scratch, the kernel
  // exchanges them; `recv_counts` (p int64, device) receives what arrived.
  void alltoallv_dev(uint64_t in, uint64_t counts, uint64_t out, uint64_t out_elems, uint64_t recv_counts,
                     int elem_bytes, uint64_t stream, int max_blocks);
  void alltoall(uint64_t in, uint64_t out, uint64_t bytes_per_peer, uint64_t stream, int max_blocks,
                bool symmetric, int mode = 0);
  // mode A2A_PUSH: symmetric buffers only, the root writes into every peer's buffer
  void bcast(uint64_t buf, uint64_t nbytes, int root, uint64_t stream, int max_blocks, bool symmetric, int mode = 0);
  void local_reduce(const std::vector<uint64_t>& ins, uint64_t out, uint64_t count, int dtype, int op,
                    uint64_t stream);
  // TP layout-fused collectives: rows x k shards <-> rows x p*k (last axis)
  void allgather_lastaxis(uint64_t in, uint64_t out, uint64_t rows, uint64_t row_bytes, uint64_t stream,
                          int max_blocks, bool symmetric);
  void reduce_scatter_lastaxis(uint64_t in, uint64_t out, uint64_t rows, uint64_t k, int dtype, int op,
                               uint64_t stream, int max_blocks, bool symmetric);

  // ---- RCCL (vendor library: baseline + P2P transport) ---------------------
  static std::string rccl_unique_id();
  void rccl_init(const std::string& uid);
  // best-effort ncclCommRegister of every symmetric segment (zero-copy RCCL
  // collectives on them); returns how many segments are registered
  int rccl_register_segments();
  // collective over the PARENT's RCCL comm (every parent rank calls; color < 0 = not a member)
  void rccl_split_from(DeviceComm* parent, int color, int key);
  static void rccl_split_leave(DeviceComm* parent);
  bool rccl_ready() const { return nccl_ != nullptr; }
  void rccl_allreduce(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, uint64_t stream);
  void rccl_reduce_scatter(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, uint64_t stream);
  void rccl_allgather(uint64_t in, uint64_t out, uint64_t count, int dtype, uint64_t stream);
  void rccl_alltoall(uint64_t in, uint64_t out, uint64_t count, int dtype, uint64_t stream);
  void rccl_bcast(uint64_t buf, uint64_t count, int dtype, int root, uint64_t stream);
  // reference myAlltoall2 rounds as grouped RCCL send/recv (the library form of algo="pairwise")
  void p2p_pairwise_alltoall(uint64_t in, uint64_t out, uint64_t bytes_per_peer, uint64_t stream);

  // ---- row-parallel GEMM with the TP all-reduce fused into its epilogue ------
  // (gemm_common.hpp FusedState).  Setup, collective through the Python layer:
  // fused_alloc() returns this rank's IPC handle, fused_connect() maps the peers'.
  std::string fused_alloc();
  void fused_connect(const std::vector<std::string>& handles);
  // the symmetric inbox (a heap block on every rank) and every rank's code of it
  void set_fused_inbox(uint64_t ptr, uint64_t bytes, const std::vector<uint64_t>& codes);
  uint64_t fused_inbox_bytes() const { return fused_inbox_bytes_; }
  // out[M, N] = sum over the group of A_r[M, K_r] . B_r[N, K_r]^T (+ bias), bf16; `out`
  // registered (heap or on-demand) on every rank, 16-B aligned, N % 8 == 0
  void gemm_rowpar(uint64_t A, uint64_t B, uint64_t out, uint64_t bias, int M, int N, int K, int lda, int ldb,
                   int ldc, float alpha, int bias_kind, uint64_t stream);
  // Push row-parallel GEMM: out[M, N] = sum over the group of A_r . B_r^T (bf16, no bias).
  // Each rank's GEMM epilogue stores its partial of row block j (M / p rows) straight into
  // rank j's slot [rank] of `inbox` (a symmetric heap block of M * N * 2 bytes on every
  // rank), then one inbox-to-local two-shot reduces the slots and pulls every block into
  // `out` (any local 16-B aligned tensor).  M % (256 p) == 0, K % 64 == 0, N % 8 == 0.
  void gemm_push_rowpar(uint64_t A, uint64_t B, uint64_t out, uint64_t inbox, int M, int N, int K, int lda, int ldb,
                        float alpha, uint64_t stream, int max_blocks);
  // The two halves of any push row-parallel producer (a GEMM epilogue, the harness's
  // attention + per-token fc_o kernel): push_targets() = where THIS rank's partial of row
  // block j goes -- rank j's slot [rank] of `inbox` (peer-mapped addresses, p of them; `inbox`
  // a symmetric heap block of nbytes on every rank, nbytes % (16 p) == 0); inbox_to_local()
  // = the collective that follows the producer on the same stream: every rank reduces its
  // p slots in rank order and pulls every reduced block into `out` (a local tensor).
  std::vector<uint64_t> push_targets(uint64_t inbox, uint64_t nbytes);
  void inbox_to_local(uint64_t inbox, uint64_t out, uint64_t nbytes, int dtype, uint64_t stream, int max_blocks);
  // TP sum of pushed per-token rows + mean over each group of `rows` rows, fanned out to every
  // rank's `out` (symmetric, nbytes / rows bytes): the fused-fc_o logits (k_inbox_mean)
  void inbox_mean(uint64_t inbox, uint64_t out, uint64_t nbytes, int rows, uint64_t stream, int max_blocks);
  uint64_t code_of_public(uint64_t ptr, uint64_t nbytes) const { return code_of_(ptr, nbytes); }
  bool fused_ready() const { return fused_tab_dev_ != nullptr && fused_inbox_bytes_ > 0; }

  // ---- health ------------------------------------------------------------
  uint32_t error_code();  // synchronises; 0 = ok
  uint32_t poll_error() const;  // non-blocking read of the host-mapped mirror (watchdog)
  void clear_error();
  // zero flags + epochs (call on every rank between host barriers, no kernel in flight)
  void reset_state();
  // symmetric inbox for the push two-shot all-reduce (>= p shards)
  void set_inbox(uint64_t ptr, uint64_t bytes);
  // LL (low-latency) all-reduce buffers: 2 parities x p sources x (2 * max_bytes)
  // of uncached device memory per rank.  ll_alloc returns this rank's IPC handle;
  // ll_connect maps every peer's (collective bootstrap by the Python layer).
  std::string ll_alloc(uint64_t max_bytes);
  void ll_connect(const std::vector<std::string>& handles);
  uint64_t ll_max_bytes() const { return ll_ready_ ? ll_max_ : 0; }
  uint64_t inbox_bytes() const { return inbox_bytes_; }
  uint64_t timeout_ticks() const { return timeout_ticks_; }
  void set_timeout_seconds(double s) { timeout_ticks_ = (uint64_t)(s * 1e8); }
  void set_copy_engine(bool on) { copy_engine_ = on; }
  // concurrent rings of the ring all-reduce (coprime strides, at most kMaxRings)
  void set_rings(int r) { rings_ = std::max(1, r); }
  void set_debug_stamps(uint64_t ptr) { dbg_ = reinterpret_cast<uint64_t*>(ptr); }  // LL kernel phase stamps
  int rings() const { return rings_; }
  // inbox bytes per chunk slot of the ring / rhd all-reduce of `nbytes` over p ranks
  static uint64_t ring_slot_bytes(uint64_t nbytes, int p);

 private:
  void sync_table_();
  void alltoall_pairwise_(uint64_t in, uint64_t out, uint64_t bytes_per_peer, hipStream_t st, int max_blocks,
                          bool symmetric);
  void allreduce_ll_(uint64_t in, uint64_t out, uint64_t nbytes, int dtype, int op, hipStream_t st, int max_blocks);
  void allreduce_pipelined_(int algo, uint64_t in, uint64_t out, uint64_t nbytes, uint64_t es, int dtype, int op,
                            hipStream_t st, int max_blocks, bool symmetric);
  CollArgs args_(uint64_t src_code, uint64_t res_code, char* out, uint64_t nbytes, int root) const;
  int grid_(uint64_t work_bytes, int max_blocks) const;
  uint64_t code_of_(uint64_t ptr, uint64_t nbytes) const;  // 0 if not registered / misaligned
  // true while a collective whose caller passed symmetric=true runs: its tensors are
  // heap blocks or were registered on demand for this call, so on-demand slots may
  // resolve them; any other call (staging paths included) sees heap segments only
  bool search_dynamic_ = false;
  struct DynScope {
    DeviceComm* d;
    DynScope(DeviceComm* c, bool on) : d(c) { d->search_dynamic_ = on; }
    ~DynScope() { d->search_dynamic_ = false; }
  };

  int rank_, size_, device_;
  Signals* sig_ = nullptr;               // mine (uncached)
  std::vector<Signals*> peer_sig_;       // mapped (mine at [rank_])
  std::vector<SegInfo> segs_;            // [0] = scratch
  std::vector<std::vector<char*>> peer_seg_;  // [seg][rank]
  PeerTable host_pt_{};
  uint32_t* host_err_ = nullptr;         // pinned, device-mapped timeout mirror
  std::vector<void*> rccl_regs_;         // ncclCommRegister handles, one per registered segment
  uint64_t chunk_cap_ = 0;               // CCMPI_CHUNK_BYTES: cap on staging chunks (0 = scratch-sized)
  uint64_t staging_chunk_(uint64_t budget, uint64_t align) const;
  PeerTable* dev_pt_ = nullptr;
  uint64_t* epochs_ = nullptr;
  uint64_t timeout_ticks_ = 2000000000ull;  // 20 s
  ncclComm_t nccl_ = nullptr;
  uint64_t inbox_ptr_ = 0, inbox_bytes_ = 0;
  uint64_t ll_max_ = 0;
  char* ll_buf_ = nullptr;                // mine (uncached)
  bool ll_ready_ = false;
  uint32_t* ll_state_ = nullptr;          // [epoch, finished CTAs] of the LL kernel
  int rings_ = 1;
  uint64_t* dbg_ = nullptr;
  bool copy_engine_ = false;              // single-rank copies: contiguous-slice kernel (3.2 vs 2.6 TB/s for the runtime blit)
  std::vector<std::string> opened_;      // handles we opened (for release)
  std::vector<std::vector<std::string>> seg_keys_;  // per slot: IPC keys opened for on-demand segments
  gemm::FusedState* fused_state_ = nullptr;  // mine (uncached)
  gemm::FusedTable fused_tab_{};            // host copy
  gemm::FusedTable* fused_tab_dev_ = nullptr;
  uint64_t fused_inbox_bytes_ = 0;
  uint64_t fused_seq_ = 0;
};

// Process-wide registry so a handle opened by two communicators maps once.
void* ipc_open(const std::string& handle, const std::string& key = std::string());
void ipc_close(const std::string& handle);

}  // namespace dev
}  // namespace ccmpi
