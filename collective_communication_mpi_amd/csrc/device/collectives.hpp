// Host-visible interface of the hand-written collective kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace ccmpi {
namespace dev {

enum AllreduceAlgo : int {
  ALGO_ONESHOT = 0,       // every rank reads everything (small messages)
  ALGO_TWOSHOT = 1,       // reduce-scatter + all-gather over all links (large)
  ALGO_REDUCE_BCAST = 2,  // reference algorithm: reduce to root, broadcast
  ALGO_TWOSHOT_PUSH = 3,  // two-shot with remote writes (scatter into peers' inboxes, push results)
  ALGO_RING = 4,          // pipelined ring RS + AG with peer writes, several rings (coprime strides)
  ALGO_RHD = 5,           // recursive halving (RS) + doubling (AG) with peer writes, p = 2^k
  ALGO_LL = 6,            // low-latency one-shot: (data, flag) 8-B units pushed to every peer, no barriers
  ALGO_TWOSHOT_FANOUT = 7,  // one phase: pull-reduce my shard, store it into every rank's result (posted writes)
  ALGO_TWOSHOT_FANOUT_LDS = 8,  // the same, peer vectors staged through LDS by DMA (no VGPRs held in flight)
};

enum MoveMode : int {
  MOVE_ALLGATHER = 0,     // pull: out[j] <- in_j
  MOVE_ALLTOALL = 1,      // pull: out[j] <- in_j[me]
  MOVE_BCAST = 2,         // pull: out <- in_root
  MOVE_ALLTOALL_PUSH = 3,  // push: out_j[me] <- in[j]  (peer writes, input stays local)
  MOVE_ALLGATHER_PUSH = 4,  // push: out_j[me] <- in     (peer writes, input stays local)
  MOVE_BCAST_PUSH = 5       // push: out_j <- in_root    (the root's CTAs fan each vector out)
};

constexpr int kMaxRings = 8;
enum AlltoallMode : int { A2A_PULL = 0, A2A_PUSH = 1, A2A_PAIRWISE = 2 };

struct CollArgs {
  const PeerTable* pt;     // device-resident peer table
  uint64_t* epochs;        // per-CTA epoch counters (device, local)
  uint64_t src_code;       // this rank's published input  (addr_code)
  uint64_t res_code;       // this rank's published result buffer (two-shot / reduce_bcast / ring / rhd / push)
  char* out;               // local output pointer (16-B aligned)
  uint64_t nbytes;         // see each kernel
  uint64_t timeout_ticks;  // bounded spins, 100 MHz ticks
  int root;
  int nrings;              // ring: number of concurrent rings (CTA b runs ring b % nrings)
  uint64_t flags;          // k_move bit 0: peer-major CTA mapping (CTA b moves only peer b % p's block)
  const char* in;          // local input (push two-shot / ring / rhd / push all-to-all read only their own input;
                           // those kernels publish the inbox in src_code instead)
  uint64_t src_stride;     // all-to-all: bytes between per-peer blocks of the source (0 = nbytes)
  uint64_t dst_stride;     // all-to-all: bytes between per-peer blocks of the destination (0 = nbytes)
  uint64_t inbox_slot;     // ring / rhd: bytes per inbox chunk slot (>= the largest chunk, 16-B multiple)
  int8_t ring_stride[kMaxRings];  // ring k: i -> i + stride (coprime to p)
  int8_t ring_inv[kMaxRings];     // stride^-1 mod p: position of rank r in ring k = r * inv % p
  uint32_t* ll_state;      // LL all-reduce: [0] call epoch, [1] finished-CTA count (device, local)
  uint64_t ll_slot;        // LL all-reduce: bytes of one (parity, source) region of the LL buffer
  uint64_t* dbg;           // optional: per-phase s_memrealtime stamps of CTA 0 / thread 0 (diagnostics)
};

// All-to-all with per-peer sizes (push): bytes [soff[j], soff[j] + len[j]) of the
// local input go to peer j's registered output at doff[j].  a.nbytes = this rank's
// total send bytes; every offset and length is a multiple of 16 B.
struct VArgs {
  CollArgs a;
  uint64_t soff[kMaxRanks];
  uint64_t doff[kMaxRanks];
  uint64_t len[kMaxRanks];
};

// Ragged all-to-all with the counts on the device (no host round trip; graph
// capturable): every rank's row [count to rank 0 .. count to rank p-1, output
// capacity in elements] (p + 1 int64) lives at the start of its scratch segment:
// the counts copied there before the kernel, the capacity written by the kernel.
struct VDevArgs {
  CollArgs a;                // src_code = scratch (segment 0) code, res_code = output code
  int64_t* recv_counts;      // out: elements received from each rank
  uint32_t es;               // element size in bytes
  int64_t cap;               // this rank's output capacity in elements (written into its row)
};

struct LocalReduceArgs {
  const char* in[kMaxRanks];
  char* out;
  uint64_t nbytes;
  int n_in;
  int pad;
};

int grid_for(uint64_t bytes_per_cta_work, int max_blocks);
void launch_copy(const void* src, void* dst, uint64_t nbytes, hipStream_t s);
void launch_allreduce(int algo, const CollArgs& a, int nranks, int dtype, int op, int grid, hipStream_t s);
// the collective half of the push row-parallel GEMM: reduce the inbox slots the GEMM
// epilogues filled (codes[0] = the inboxes), pull every shard into a.out (bf16 / fp32 sum)
void launch_inbox_to_local(const CollArgs& a, int nranks, int dtype, int grid, hipStream_t s);
void launch_inbox_mean(const CollArgs& a, int nranks, int grid, hipStream_t s);
void launch_reduce_scatter(const CollArgs& a, int nranks, int dtype, int op, int grid, hipStream_t s);
void launch_move(int mode, const CollArgs& a, int nranks, int grid, hipStream_t s);
// mode 0: last-axis all-gather, 1: last-axis reduce-scatter; rows passed in CollArgs::root
void launch_lastaxis(int mode, const CollArgs& a, int nranks, int dtype, int op, int grid, hipStream_t s);
void launch_local_reduce(const LocalReduceArgs& a, int dtype, int op, hipStream_t s);
void launch_alltoallv(const VArgs& v, int grid, hipStream_t s);
// pairwise rounds (push, one peer per round): a.in local input, a.res_code the
// registered output (or scratch), nbytes per block, src/dst strides as k_move
void launch_alltoall_pairwise(const CollArgs& a, int grid, hipStream_t s);
void launch_alltoallv_dev(const VDevArgs& v, int grid, hipStream_t s);

}  // namespace dev
}  // namespace ccmpi
