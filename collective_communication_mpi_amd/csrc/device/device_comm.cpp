// Device communicator implementation (host code; kernels in collectives.hip).
#include "device_comm.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace ccmpi {
namespace dev {

namespace {

std::mutex g_ipc_mu;
std::map<std::string, std::pair<void*, int>> g_ipc;  // handle bytes -> (base, refs)

ncclDataType_t nccl_dt(int dt) {
  switch (dt) {
    case DT_I8: return ncclInt8;
    case DT_U8: case DT_BOOL: case DT_BYTE: return ncclUint8;
    case DT_I32: return ncclInt32;
    case DT_U32: return ncclUint32;
    case DT_I64: return ncclInt64;
    case DT_U64: return ncclUint64;
    case DT_F16: return ncclFloat16;
    case DT_BF16: return ncclBfloat16;
    case DT_F32: return ncclFloat32;
    case DT_F64: return ncclFloat64;
  }
  throw std::invalid_argument("ccmpi: dtype unsupported by RCCL: " + std::to_string(dt));
}

ncclRedOp_t nccl_op(int op) {
  switch (op) {
    case OP_SUM: return ncclSum;
    case OP_PROD: return ncclProd;
    case OP_MIN: return ncclMin;
    case OP_MAX: return ncclMax;
  }
  throw std::invalid_argument("ccmpi: op unsupported by RCCL: " + std::to_string(op));
}

#define CCMPI_NCCL_CHECK(expr)                                                                   \
  do {                                                                                            \
    ncclResult_t _r = (expr);                                                                     \
    if (_r != ncclSuccess)                                                                        \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " #expr); \
  } while (0)

inline hipStream_t S(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

void* ipc_open(const std::string& handle, const std::string& key_in) {
  const std::string& key = key_in.empty() ? handle : key_in;
  std::lock_guard<std::mutex> g(g_ipc_mu);
  auto it = g_ipc.find(key);
  if (it != g_ipc.end()) {
    it->second.second++;
    return it->second.first;
  }
  if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("ccmpi: bad IPC handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  CCMPI_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  g_ipc[key] = {p, 1};
  return p;
}

void ipc_close(const std::string& handle) {
  std::lock_guard<std::mutex> g(g_ipc_mu);
  auto it = g_ipc.find(handle);
  if (it == g_ipc.end()) return;
  if (--it->second.second == 0) {
    (void)hipIpcCloseMemHandle(it->second.first);
    g_ipc.erase(it);
  }
}

DeviceComm::DeviceComm(int rank, int size, int device, uint64_t /*scratch_bytes*/)
    : rank_(rank), size_(size), device_(device) {
  if (size < 1 || size > kMaxRanks) throw std::invalid_argument("ccmpi: device communicator supports 1..16 ranks");
  CCMPI_HIP_CHECK(hipSetDevice(device));
  CCMPI_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sizeof(Signals), hipDeviceMallocUncached));
  CCMPI_HIP_CHECK(hipMemset(sig_, 0, sizeof(Signals)));
  CCMPI_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&epochs_), sizeof(uint64_t) * kMaxBlocks));
  CCMPI_HIP_CHECK(hipMemset(epochs_, 0, sizeof(uint64_t) * kMaxBlocks));
  CCMPI_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&dev_pt_), sizeof(PeerTable)));
  CCMPI_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&ll_state_), 2 * sizeof(uint32_t)));
  CCMPI_HIP_CHECK(hipMemset(ll_state_, 0, 2 * sizeof(uint32_t)));
  std::memset(&host_pt_, 0, sizeof(host_pt_));
  host_pt_.rank = rank;
  host_pt_.size = size;
  peer_sig_.assign(size, nullptr);
  peer_sig_[rank] = sig_;
  host_pt_.sig[rank] = sig_;
  CCMPI_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_err_), sizeof(uint32_t),
                                hipHostMallocMapped | hipHostMallocCoherent));
  *host_err_ = 0;
  CCMPI_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_pt_.host_err), host_err_, 0));
  if (const char* t = std::getenv("CCMPI_DEVICE_TIMEOUT_S")) set_timeout_seconds(std::atof(t));
  if (const char* c = std::getenv("CCMPI_COPY_ENGINE")) copy_engine_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("CCMPI_CHUNK_BYTES")) chunk_cap_ = std::strtoull(c, nullptr, 10);
  CCMPI_HIP_CHECK(hipDeviceSynchronize());
  sync_table_();
}

DeviceComm::~DeviceComm() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (void* h : rccl_regs_)
    if (nccl_ && h) ncclCommDeregister(nccl_, h);
  if (nccl_) ncclCommDestroy(nccl_);
  for (auto& h : opened_) ipc_close(h);
  for (auto& ks : seg_keys_)
    for (auto& k : ks) ipc_close(k);
  if (sig_) (void)hipFree(sig_);
  if (epochs_) (void)hipFree(epochs_);
  if (dev_pt_) (void)hipFree(dev_pt_);
  if (ll_state_) (void)hipFree(ll_state_);
  if (ll_buf_) (void)hipFree(ll_buf_);
  if (fused_state_) (void)hipFree(fused_state_);
  if (fused_tab_dev_) (void)hipFree(fused_tab_dev_);
  if (host_err_) (void)hipHostFree(host_err_);
}

void DeviceComm::sync_table_() {
  CCMPI_HIP_CHECK(hipMemcpy(dev_pt_, &host_pt_, sizeof(PeerTable), hipMemcpyHostToDevice));
}

std::string DeviceComm::signal_handle() const {
  hipIpcMemHandle_t h;
  CCMPI_HIP_CHECK(hipIpcGetMemHandle(&h, sig_));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void DeviceComm::connect(const std::vector<std::string>& sig_handles) {
  if ((int)sig_handles.size() != size_) throw std::invalid_argument("ccmpi: need one signal handle per rank");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  for (int j = 0; j < size_; ++j) {
    if (j == rank_) continue;
    void* p = ipc_open(sig_handles[j]);
    opened_.push_back(sig_handles[j]);
    peer_sig_[j] = static_cast<Signals*>(p);
    host_pt_.sig[j] = peer_sig_[j];
  }
  sync_table_();
}

std::pair<std::string, uint64_t> DeviceComm::export_range(uint64_t ptr) const {
  hipDeviceptr_t base = nullptr;
  size_t sz = 0;
  CCMPI_HIP_CHECK(hipMemGetAddressRange(&base, &sz, reinterpret_cast<hipDeviceptr_t>(ptr)));
  hipIpcMemHandle_t h;
  CCMPI_HIP_CHECK(hipIpcGetMemHandle(&h, base));
  return {std::string(reinterpret_cast<const char*>(&h), sizeof(h)), ptr - (uint64_t)base};
}

int DeviceComm::add_segment(uint64_t local_ptr, uint64_t bytes, const std::vector<std::string>& handles,
                            const std::vector<uint64_t>& offsets) {
  if ((int)segs_.size() >= kMaxSegs) throw std::runtime_error("ccmpi: too many symmetric segments");
  if ((int)handles.size() != size_ || (int)offsets.size() != size_)
    throw std::invalid_argument("ccmpi: add_segment needs one handle per rank");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  const int s = (int)segs_.size();
  segs_.push_back(SegInfo{reinterpret_cast<char*>(local_ptr), bytes, false});
  peer_seg_.emplace_back(size_, nullptr);
  for (int j = 0; j < size_; ++j) {
    char* p;
    if (j == rank_) {
      p = reinterpret_cast<char*>(local_ptr);
    } else {
      p = static_cast<char*>(ipc_open(handles[j])) + offsets[j];
      opened_.push_back(handles[j]);
    }
    peer_seg_[s][j] = p;
    host_pt_.seg[j][s] = p;
  }
  host_pt_.seg_bytes[s] = bytes;
  host_pt_.nsegs = (int)segs_.size();
  sync_table_();
  return s;
}

// On-demand registration of an ordinary allocation (torch caching-allocator segment):
// slot `s` (-1 = a new slot) maps every rank's allocation; `keys[j]` identifies rank j's
// allocation generation (the IPC handle bytes plus the owner's allocator generation),
// so a freed-and-reallocated segment at the same address is opened afresh.  The
// previous occupant's peer mappings are released (the caller has synchronised the
// device: no kernel of this rank still resolves through the slot).
int DeviceComm::set_segment(int s, uint64_t local_ptr, uint64_t bytes, const std::vector<std::string>& handles,
                            const std::vector<uint64_t>& offsets, const std::vector<std::string>& keys) {
  if ((int)handles.size() != size_ || (int)offsets.size() != size_ || (int)keys.size() != size_)
    throw std::invalid_argument("ccmpi: set_segment needs one handle/offset/key per rank");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  if (s < 0) {
    if ((int)segs_.size() >= kMaxSegs) throw std::runtime_error("ccmpi: too many registered segments");
    s = (int)segs_.size();
    segs_.push_back(SegInfo{});
    peer_seg_.emplace_back(size_, nullptr);
    seg_keys_.resize(segs_.size());
  } else if (s == 0 || s >= (int)segs_.size()) {
    throw std::invalid_argument("ccmpi: set_segment: bad slot");
  }
  seg_keys_.resize(segs_.size());
  for (auto& k : seg_keys_[s]) ipc_close(k);
  seg_keys_[s].clear();
  segs_[s] = SegInfo{reinterpret_cast<char*>(local_ptr), bytes, false, true};
  for (int j = 0; j < size_; ++j) {
    char* p;
    if (j == rank_) {
      p = reinterpret_cast<char*>(local_ptr);
    } else {
      p = static_cast<char*>(ipc_open(handles[j], keys[j])) + offsets[j];
      seg_keys_[s].push_back(keys[j]);
    }
    peer_seg_[s][j] = p;
    host_pt_.seg[j][s] = p;
  }
  host_pt_.seg_bytes[s] = bytes;
  host_pt_.nsegs = (int)segs_.size();
  sync_table_();
  return s;
}

void DeviceComm::clear_segment(int s) {
  if (s <= 0 || s >= (int)segs_.size()) throw std::invalid_argument("ccmpi: clear_segment: bad slot");
  seg_keys_.resize(segs_.size());
  for (auto& k : seg_keys_[s]) ipc_close(k);
  seg_keys_[s].clear();
  segs_[s] = SegInfo{nullptr, 0, false, true};  // local range empty: find() never matches it
  for (int j = 0; j < size_; ++j) {
    peer_seg_[s][j] = nullptr;
    host_pt_.seg[j][s] = nullptr;
  }
  host_pt_.seg_bytes[s] = 0;
  sync_table_();
}

int DeviceComm::find(uint64_t ptr, uint64_t nbytes, uint64_t* off, bool dynamic) const {
  for (size_t s = 0; s < segs_.size(); ++s) {
    if (segs_[s].dynamic && !dynamic) continue;
    uint64_t b = (uint64_t)segs_[s].local;
    if (ptr >= b && ptr + nbytes <= b + segs_[s].bytes) {
      if (off) *off = ptr - b;
      return (int)s;
    }
  }
  return -1;
}

uint64_t DeviceComm::code_of_(uint64_t ptr, uint64_t nbytes) const {
  if (ptr % 16) return 0;
  uint64_t off = 0;
  int s = find(ptr, nbytes, &off, search_dynamic_);
  if (s < 0) return 0;
  return addr_code(s, off);
}

CollArgs DeviceComm::args_(uint64_t src_code, uint64_t res_code, char* out, uint64_t nbytes, int root) const {
  CollArgs a{};
  a.pt = dev_pt_;
  a.epochs = epochs_;
  a.src_code = src_code;
  a.res_code = res_code;
  a.out = out;
  a.nbytes = nbytes;
  a.timeout_ticks = timeout_ticks_;
  a.root = root;
  return a;
}

int DeviceComm::grid_(uint64_t work_bytes, int max_blocks) const {
  if (max_blocks <= 0) max_blocks = 256;
  return grid_for(work_bytes, std::min(max_blocks, kMaxBlocks));
}

void DeviceComm::allreduce(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, int algo,
                           uint64_t stream, int max_blocks, bool symmetric) {
  DynScope dyn_scope(this, symmetric);
  const uint64_t es = dtype_bytes(dtype), nbytes = count * es;
  if (!device_reduce_supported(dtype, op)) throw std::invalid_argument("ccmpi: unsupported device reduction");
  if (nbytes == 0) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (size_ == 1) {
    if (in != out) {
      if (copy_engine_) CCMPI_HIP_CHECK(hipMemcpyAsync((void*)out, (void*)in, nbytes, hipMemcpyDeviceToDevice, st));
      else launch_copy((const void*)in, (void*)out, nbytes, st);
    }
    return;
  }
  if (algo == ALGO_LL) {
    // global decision (sizes and the LL setup are identical on every rank)
    if (ll_ready_ && nbytes % 16 == 0 && nbytes <= ll_max_) {
      allreduce_ll_(in, out, nbytes, dtype, op, st, max_blocks);
      return;
    }
    algo = ALGO_ONESHOT;
  }
  if (algo == ALGO_RING || algo == ALGO_RHD) {
    allreduce_pipelined_(algo, in, out, nbytes, es, dtype, op, st, max_blocks, symmetric);
    return;
  }
  if (algo == ALGO_TWOSHOT_PUSH) {
    // needs registered in/out and an inbox of p shards; otherwise the pull form
    const uint64_t shard = ((nbytes + size_ - 1) / size_ + 15) / 16 * 16;
    const uint64_t ic = inbox_ptr_ ? code_of_(inbox_ptr_, inbox_bytes_) : 0;
    uint64_t sc = code_of_(in, nbytes), rc = code_of_(out, nbytes);
    if (symmetric && sc && rc && ic && in != out && inbox_bytes_ >= shard * size_) {
      CollArgs a = args_(ic, rc, (char*)out, nbytes, 0);  // the inbox is published in slot 0
      a.in = reinterpret_cast<const char*>(in);
      launch_allreduce(ALGO_TWOSHOT_PUSH, a, size_, dtype, op, grid_(nbytes / size_, max_blocks), st);
      return;
    }
    algo = ALGO_TWOSHOT;
  }
  const bool needs_res = algo != ALGO_ONESHOT;
  // the fan-out kernel stores every shard into the ranks' result buffers
  // (codes[1]) and never touches `out` itself: a staged result is copied back
  const bool fan = algo == ALGO_TWOSHOT_FANOUT || algo == ALGO_TWOSHOT_FANOUT_LDS;
  const bool sharded = algo == ALGO_TWOSHOT || fan;
  if (symmetric && !(algo == ALGO_ONESHOT && in == out)) {
    uint64_t sc = code_of_(in, nbytes), rc = needs_res ? code_of_(out, nbytes) : 0;
    if (!sc || (needs_res && !rc) || out % 16)
      throw std::invalid_argument("ccmpi: symmetric allreduce needs 16-B aligned registered buffers");
    const uint64_t work = sharded ? nbytes / size_ : nbytes;
    launch_allreduce(algo, args_(sc, rc, (char*)out, nbytes, 0), size_, dtype, op, grid_(work, max_blocks), st);
    return;
  }
  if (scratch_bytes() < 64 * es) throw std::runtime_error("ccmpi: scratch segment missing or too small");
  // chunk size identical on all ranks: half the scratch, 16-B and element aligned
  uint64_t chunk = staging_chunk_(scratch_bytes() / 2, 16 * es);
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  for (uint64_t off = 0; off < nbytes; off += chunk) {
    const uint64_t n = std::min(chunk, nbytes - off);
    uint64_t sc = (algo == ALGO_ONESHOT && in == out) ? 0 : code_of_(in + off, n);
    if (!sc) {
      CCMPI_HIP_CHECK(hipMemcpyAsync(stage, (void*)(in + off), n, hipMemcpyDeviceToDevice, st));
      sc = addr_code(0, 0);
    }
    const bool out_ok = (out + off) % 16 == 0;
    uint64_t rc = 0;
    char* outp = (char*)(out + off);
    bool res_staged = false;
    if (needs_res) {
      rc = out_ok ? code_of_(out + off, n) : 0;
      if (!rc) {
        rc = addr_code(0, chunk);
        res_staged = fan;
      }
    }
    if (!out_ok) outp = stage + chunk;
    const uint64_t work = sharded ? n / size_ : n;
    launch_allreduce(algo, args_(sc, rc, outp, n, 0), size_, dtype, op, grid_(work, max_blocks), st);
    if (!out_ok || res_staged)
      CCMPI_HIP_CHECK(hipMemcpyAsync((void*)(out + off), stage + chunk, n, hipMemcpyDeviceToDevice, st));
  }
}

void DeviceComm::allreduce_to_local(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, uint64_t stream,
                                    int max_blocks) {
  const uint64_t es = dtype_bytes(dtype), nbytes = count * es;
  if (!device_reduce_supported(dtype, op)) throw std::invalid_argument("ccmpi: unsupported device reduction");
  if (nbytes == 0) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (size_ == 1) {
    if (in != out) launch_copy((const void*)in, (void*)out, nbytes, st);
    return;
  }
  const uint64_t sc = code_of_(in, nbytes);
  if (!sc || out % 16 || in == out)
    throw std::invalid_argument("ccmpi: allreduce_to_local needs a 16-B aligned symmetric source and a distinct 16-B "
                                "aligned output");
  // res = src: the reduce-scatter writes shard r into rank r's own source, the
  // all-gather reads every rank's source shard into the local output
  launch_allreduce(ALGO_TWOSHOT, args_(sc, sc, (char*)out, nbytes, 0), size_, dtype, op, grid_(nbytes / size_, max_blocks),
                   st);
}

void DeviceComm::allreduce_ll_(uint64_t in, uint64_t out, uint64_t nbytes, int dtype, int op, hipStream_t st,
                               int max_blocks) {
  // misaligned local buffers go through the scratch segment (local copies only:
  // the protocol is the same on every rank)
  const char* inp = reinterpret_cast<const char*>(in);
  char* outp = reinterpret_cast<char*>(out);
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  if (in % 16) {
    CCMPI_HIP_CHECK(hipMemcpyAsync(stage, inp, nbytes, hipMemcpyDeviceToDevice, st));
    inp = stage;
  }
  const bool out_staged = out % 16 != 0;
  if (out_staged) outp = stage + scratch_bytes() / 2 / 16 * 16;
  CollArgs a = args_(0, 0, outp, nbytes, 0);
  a.in = inp;
  a.ll_state = ll_state_;
  a.dbg = dbg_;
  a.ll_slot = 2 * ll_max_;
  const uint64_t nvec = nbytes / 16;
  int g = (int)std::min<uint64_t>((nvec + 255) / 256, (uint64_t)std::max(1, std::min(max_blocks, kMaxBlocks)));
  launch_allreduce(ALGO_LL, a, size_, dtype, op, std::max(g, 1), st);
  if (out_staged) CCMPI_HIP_CHECK(hipMemcpyAsync((void*)out, outp, nbytes, hipMemcpyDeviceToDevice, st));
}

std::string DeviceComm::ll_alloc(uint64_t max_bytes) {
  if (ll_buf_) throw std::runtime_error("ccmpi: LL buffers already allocated");
  if (max_bytes == 0 || max_bytes % 16) throw std::invalid_argument("ccmpi: LL max bytes must be a positive multiple of 16");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  const uint64_t bytes = 2ull * size_ * 2 * max_bytes;
  CCMPI_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&ll_buf_), bytes, hipDeviceMallocUncached));
  CCMPI_HIP_CHECK(hipMemset(ll_buf_, 0, bytes));
  CCMPI_HIP_CHECK(hipDeviceSynchronize());
  ll_max_ = max_bytes;
  hipIpcMemHandle_t h;
  CCMPI_HIP_CHECK(hipIpcGetMemHandle(&h, ll_buf_));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void DeviceComm::ll_connect(const std::vector<std::string>& handles) {
  if (!ll_buf_ || (int)handles.size() != size_) throw std::invalid_argument("ccmpi: ll_connect needs ll_alloc and one handle per rank");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  for (int j = 0; j < size_; ++j) {
    if (j == rank_) {
      host_pt_.ll[j] = ll_buf_;
      continue;
    }
    host_pt_.ll[j] = static_cast<char*>(ipc_open(handles[j]));
    opened_.push_back(handles[j]);
  }
  sync_table_();
  ll_ready_ = true;
}

namespace {
int gcd_i(int a, int b) { return b ? gcd_i(b, a % b) : a; }
int inv_mod(int a, int m) {
  for (int x = 1; x < m; ++x)
    if ((a * x) % m == 1) return x;
  return 1;
}
}  // namespace

uint64_t DeviceComm::ring_slot_bytes(uint64_t nbytes, int p) {
  // largest part16 chunk of nbytes over p ranks
  const uint64_t nv = (nbytes + 15) / 16;
  return ((nv + p - 1) / p) * 16;
}

// `symmetric` (identical on every rank): every rank's output is registered and
// its input 16-B aligned, so results are pushed straight into peers' outputs, and
// pieces are bounded by the inbox alone.  Otherwise the result goes through the
// scratch segment (a misaligned input is staged too) in pieces of at most half the
// scratch.  The launch sequence therefore DEPENDS on `symmetric` once nbytes
// exceeds half the scratch: the caller must make the decision identical on all
// ranks there -- a promise, the collective registration path, or an all-gather of
// the rank-local check (DeviceGroup._symm_call does the last beyond half the scratch).
void DeviceComm::allreduce_pipelined_(int algo, uint64_t in, uint64_t out, uint64_t nbytes, uint64_t es, int dtype,
                                      int op, hipStream_t st, int max_blocks, bool symmetric) {
  const int p = size_;
  if (algo == ALGO_RHD && (p & (p - 1)))
    throw std::invalid_argument("ccmpi: recursive halving/doubling needs a power-of-two group size");
  const uint64_t ic = inbox_ptr_ ? code_of_(inbox_ptr_, inbox_bytes_) : 0;
  if (!ic) throw std::runtime_error("ccmpi: ring/rhd all-reduce needs the symmetric inbox (set_inbox)");
  // concurrent rings: strides coprime to p (s and p-s are the two directions of the same links)
  std::vector<int> strides;
  for (int s = 1; s < p && (int)strides.size() < std::min(rings_, kMaxRings); ++s)
    if (gcd_i(s, p) == 1) strides.push_back(s);
  if (strides.empty()) strides.push_back(1);
  const int R = algo == ALGO_RING ? (int)strides.size() : 1;
  // piece size: (p-1) inbox slots of the piece's largest chunk must fit; identical on all ranks
  uint64_t piece = (inbox_bytes_ / (p - 1) / 16) * 16 * p;
  const uint64_t half = scratch_bytes() / 2 / 16 * 16;
  const bool in_al = in % 16 == 0;
  if (symmetric && (!in_al || out % 16 || !code_of_(out, nbytes)))
    throw std::invalid_argument("ccmpi: symmetric ring/rhd all-reduce needs a registered output and aligned input");
  const bool out_reg = symmetric;
  // `symmetric` is identical on every rank (the Python layer decides it collectively, or the
  // caller promises it): with it nothing is staged, so the pieces are bounded by the inbox
  // alone -- a 1 GiB all-reduce is ONE launch, not 32 scratch-sized ones (64 MiB scratch on a
  // shared GPU: every launch paid the start barrier and the 2(p-1)-step pipeline fill again,
  // profiles/r5_ring).  Staged calls keep pieces of half the scratch.
  if (!symmetric) piece = std::min(piece, half);
  piece = staging_chunk_(piece, 16 * es);
  if (piece == 0) throw std::runtime_error("ccmpi: inbox/scratch too small for ring/rhd");
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  for (uint64_t off = 0; off < nbytes; off += piece) {
    const uint64_t n = std::min(piece, nbytes - off);
    const char* inp = reinterpret_cast<const char*>(in + off);
    if (!in_al) {
      CCMPI_HIP_CHECK(hipMemcpyAsync(stage, inp, n, hipMemcpyDeviceToDevice, st));
      inp = stage;
    }
    char* outp = reinterpret_cast<char*>(out + off);
    uint64_t rc = out_reg ? code_of_(out + off, n) : 0;
    if (!rc) {
      rc = addr_code(0, half);
      outp = stage + half;
    }
    CollArgs a = args_(ic, rc, outp, n, 0);  // the inbox is published in slot 0
    a.in = inp;
    a.inbox_slot = ring_slot_bytes(n, p);
    a.nrings = R;
    for (int k = 0; k < R; ++k) {
      a.ring_stride[k] = (int8_t)strides[k];
      a.ring_inv[k] = (int8_t)inv_mod(strides[k], p);
    }
    int g = grid_(n / p, max_blocks);
    g = std::max(R, g / R * R);
    launch_allreduce(algo, a, size_, dtype, op, g, st);
    if (outp != reinterpret_cast<char*>(out + off))
      CCMPI_HIP_CHECK(hipMemcpyAsync((void*)(out + off), outp, n, hipMemcpyDeviceToDevice, st));
  }
}

void DeviceComm::reduce_scatter(uint64_t in, uint64_t out, uint64_t count_per_rank, int dtype, int op,
                                uint64_t stream, int max_blocks, bool symmetric) {
  DynScope dyn_scope(this, symmetric);
  const uint64_t es = dtype_bytes(dtype), blk = count_per_rank * es;
  if (!device_reduce_supported(dtype, op)) throw std::invalid_argument("ccmpi: unsupported device reduction");
  if (blk == 0) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (size_ == 1) {
    if (in != out) CCMPI_HIP_CHECK(hipMemcpyAsync((void*)out, (void*)in, blk, hipMemcpyDeviceToDevice, st));
    return;
  }
  // the kernel reads block `me` of every rank at offset me*nbytes of the
  // published base; with chunking the staged layout is [p][chunk].
  if (symmetric) {
    uint64_t sc = code_of_(in, blk * size_);
    if (!sc || out % 16) throw std::invalid_argument("ccmpi: symmetric reduce_scatter needs aligned registered input");
    launch_reduce_scatter(args_(sc, 0, (char*)out, blk, 0), size_, dtype, op, grid_(blk, max_blocks), st);
    return;
  }
  uint64_t chunk = staging_chunk_(scratch_bytes() / 2 / size_, 16 * es);
  if (chunk == 0) throw std::runtime_error("ccmpi: scratch too small for reduce_scatter");
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  for (uint64_t off = 0; off < blk; off += chunk) {
    const uint64_t n = std::min(chunk, blk - off);
    for (int j = 0; j < size_; ++j)
      CCMPI_HIP_CHECK(hipMemcpyAsync(stage + j * n, (void*)(in + j * blk + off), n, hipMemcpyDeviceToDevice, st));
    const bool out_ok = (out + off) % 16 == 0;
    char* outp = out_ok ? (char*)(out + off) : stage + scratch_bytes() / 2;
    launch_reduce_scatter(args_(addr_code(0, 0), 0, outp, n, 0), size_, dtype, op, grid_(n, max_blocks), st);
    if (!out_ok) CCMPI_HIP_CHECK(hipMemcpyAsync((void*)(out + off), outp, n, hipMemcpyDeviceToDevice, st));
  }
}

// Peer-major CTA mapping for the pull all-gather and both all-to-alls: CTA b
// streams only peer (b % p)'s block (grid rounded to a multiple of p), one source
// and one destination stream per CTA instead of p interleaved ones.  Measured
// 6-10% faster for all-to-all and 23-31% for the pull all-gather at 256 MiB
// (profiles/r2_coll/peer_major.md); CCMPI_PEER_MAJOR=0 restores the all-peers
// mapping.  The push all-gather keeps it: one load there feeds p stores.
static void launch_move_m(int mode, CollArgs a, int p, int grid, hipStream_t st) {
  static const bool pm = [] {
    const char* e = std::getenv("CCMPI_PEER_MAJOR");
    return !(e && e[0] == '0');
  }();
  if (pm && (mode == MOVE_ALLGATHER || mode == MOVE_ALLTOALL || mode == MOVE_ALLTOALL_PUSH)) {
    a.flags |= 1;
    grid = std::max(p, grid / p * p);
  }
  launch_move(mode, a, p, grid, st);
}

void DeviceComm::allgather(uint64_t in, uint64_t out, uint64_t bytes_per_rank, uint64_t stream, int max_blocks,
                           bool symmetric, int mode) {
  DynScope dyn_scope(this, symmetric);
  if (bytes_per_rank == 0) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (size_ == 1) {
    if (in != out) CCMPI_HIP_CHECK(hipMemcpyAsync((void*)out, (void*)in, bytes_per_rank, hipMemcpyDeviceToDevice, st));
    return;
  }
  if (mode == A2A_PUSH) {
    // the protocol differs from the pull form, so this is the caller's global
    // decision: every rank passes a registered, 16-B aligned output
    const uint64_t rc = code_of_(out, bytes_per_rank * size_);
    if (!rc || in % 16 || out % 16 || bytes_per_rank % 16)
      throw std::invalid_argument("ccmpi: push allgather needs a registered 16-B aligned output and 16-B blocks");
    CollArgs a = args_(0, rc, (char*)out, bytes_per_rank, 0);
    a.in = reinterpret_cast<const char*>(in);
    launch_move(MOVE_ALLGATHER_PUSH, a, size_, grid_(bytes_per_rank * size_, max_blocks), st);
    return;
  }
  if (symmetric) {
    uint64_t sc = code_of_(in, bytes_per_rank);
    if (!sc || out % 16 || bytes_per_rank % 16) {
      if (!sc) throw std::invalid_argument("ccmpi: symmetric allgather needs an aligned registered input");
    }
    if (out % 16 == 0 && bytes_per_rank % 16 == 0) {
      launch_move_m(MOVE_ALLGATHER, args_(sc, 0, (char*)out, bytes_per_rank, 0), size_, grid_(bytes_per_rank * size_, max_blocks), st);
      return;
    }
  }
  // chunk over the per-rank block; destination blocks are strided by
  // bytes_per_rank so each chunk gathers into a [p][n] staging area first
  // unless the output layout can take it directly (n == bytes_per_rank).
  uint64_t chunk = staging_chunk_(scratch_bytes() / 2 / (size_ + 1), 16);
  if (chunk == 0) throw std::runtime_error("ccmpi: scratch too small for allgather");
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  char* gath = stage + chunk;
  for (uint64_t off = 0; off < bytes_per_rank; off += chunk) {
    const uint64_t n = std::min(chunk, bytes_per_rank - off);
    uint64_t sc = code_of_(in + off, n);
    if (!sc) {
      CCMPI_HIP_CHECK(hipMemcpyAsync(stage, (void*)(in + off), n, hipMemcpyDeviceToDevice, st));
      sc = addr_code(0, 0);
    }
    // chunks land in the strided output directly when it is 16-B aligned
    const bool direct = (out + off) % 16 == 0 && bytes_per_rank % 16 == 0;
    char* dst = direct ? (char*)(out + off) : gath;
    CollArgs a = args_(sc, 0, dst, n, 0);
    a.dst_stride = direct ? bytes_per_rank : n;
    launch_move_m(MOVE_ALLGATHER, a, size_, grid_(n * size_, max_blocks), st);
    if (!direct)
      CCMPI_HIP_CHECK(hipMemcpy2DAsync((void*)(out + off), bytes_per_rank, gath, n, n, size_, hipMemcpyDeviceToDevice, st));
  }
}

void DeviceComm::alltoall(uint64_t in, uint64_t out, uint64_t bytes_per_peer, uint64_t stream, int max_blocks,
                          bool symmetric, int mode) {
  DynScope dyn_scope(this, symmetric);
  if (bytes_per_peer == 0) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (size_ == 1) {
    if (in != out) CCMPI_HIP_CHECK(hipMemcpyAsync((void*)out, (void*)in, bytes_per_peer, hipMemcpyDeviceToDevice, st));
    return;
  }
  const uint64_t total = bytes_per_peer * size_;
  const bool aligned = in % 16 == 0 && out % 16 == 0 && bytes_per_peer % 16 == 0;
  if (mode == A2A_PAIRWISE) {
    alltoall_pairwise_(in, out, bytes_per_peer, st, max_blocks, symmetric && in != out && aligned);
    return;
  }
  if (symmetric && in != out && aligned) {
    if (mode == A2A_PUSH) {
      // every rank's OUTPUT is registered: peer writes straight into it, the input stays local
      const uint64_t rc = code_of_(out, total);
      if (!rc) throw std::invalid_argument("ccmpi: push alltoall needs a registered output on every rank");
      CollArgs a = args_(0, rc, (char*)out, bytes_per_peer, 0);
      a.in = reinterpret_cast<const char*>(in);
      launch_move_m(MOVE_ALLTOALL_PUSH, a, size_, grid_(total, max_blocks), st);
      return;
    }
    const uint64_t sc = code_of_(in, total);
    if (!sc) throw std::invalid_argument("ccmpi: symmetric alltoall needs an aligned registered input");
    launch_move_m(MOVE_ALLTOALL, args_(sc, 0, (char*)out, bytes_per_peer, 0), size_, grid_(total, max_blocks), st);
    return;
  }
  // Staged pull (in-place calls, unregistered inputs): one pack pass of this
  // chunk's p blocks into the scratch segment ([p][n]); the kernel pulls block
  // `me` of every peer's scratch straight into the strided output (no unpack
  // pass unless the output is misaligned).
  uint64_t chunk = staging_chunk_(scratch_bytes() / 2 / size_, 16);
  if (chunk == 0) throw std::runtime_error("ccmpi: scratch too small for alltoall");
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  char* gath = stage + scratch_bytes() / 2;
  for (uint64_t off = 0; off < bytes_per_peer; off += chunk) {
    const uint64_t n = std::min(chunk, bytes_per_peer - off);
    CCMPI_HIP_CHECK(hipMemcpy2DAsync(stage, n, (void*)(in + off), bytes_per_peer, n, size_, hipMemcpyDeviceToDevice, st));
    const bool direct = (out + off) % 16 == 0 && bytes_per_peer % 16 == 0;
    CollArgs a = args_(addr_code(0, 0), 0, direct ? (char*)(out + off) : gath, n, 0);
    a.src_stride = n;
    a.dst_stride = direct ? bytes_per_peer : n;
    launch_move_m(MOVE_ALLTOALL, a, size_, grid_(n * size_, max_blocks), st);
    if (!direct)
      CCMPI_HIP_CHECK(hipMemcpy2DAsync((void*)(out + off), bytes_per_peer, gath, n, n, size_, hipMemcpyDeviceToDevice, st));
  }
}

// Pairwise rounds push into every peer's output: registered outputs on every rank
// (`symmetric`, the caller's global promise) take the blocks directly; otherwise
// they land in the peers' scratch segments ([p][chunk], identical chunking on every
// rank) and a strided copy moves them out.  In place is always staged (a peer's
// block could overwrite input not yet sent).
void DeviceComm::alltoall_pairwise_(uint64_t in, uint64_t out, uint64_t bytes_per_peer, hipStream_t st,
                                    int max_blocks, bool symmetric) {
  const uint64_t total = bytes_per_peer * size_;
  if (symmetric) {
    const uint64_t rc = code_of_(out, total);
    if (!rc) throw std::invalid_argument("ccmpi: symmetric pairwise alltoall needs a registered output on every rank");
    CollArgs a = args_(0, rc, (char*)out, bytes_per_peer, 0);
    a.in = reinterpret_cast<const char*>(in);
    launch_alltoall_pairwise(a, grid_(bytes_per_peer, max_blocks), st);
    return;
  }
  uint64_t chunk = staging_chunk_(scratch_bytes() / 2 / size_, 16);
  if (chunk == 0) throw std::runtime_error("ccmpi: scratch too small for alltoall");
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  char* src = reinterpret_cast<char*>(in);
  if (in == out || in % 16) {
    // the input must stay intact until sent and be 16-B aligned: second half of scratch
    chunk = staging_chunk_(scratch_bytes() / 4 / size_, 16);
  }
  char* pack = stage + scratch_bytes() / 2;
  for (uint64_t off = 0; off < bytes_per_peer; off += chunk) {
    const uint64_t n = std::min(chunk, bytes_per_peer - off);
    CollArgs a = args_(0, addr_code(0, 0), stage, n, 0);
    if (in == out || in % 16) {
      CCMPI_HIP_CHECK(hipMemcpy2DAsync(pack, n, src + off, bytes_per_peer, n, size_, hipMemcpyDeviceToDevice, st));
      a.in = pack;
      a.src_stride = n;
    } else {
      a.in = src + off;
      a.src_stride = bytes_per_peer;
    }
    a.dst_stride = n;
    launch_alltoall_pairwise(a, grid_(n, max_blocks), st);
    CCMPI_HIP_CHECK(hipMemcpy2DAsync((void*)(out + off), bytes_per_peer, stage, n, n, size_, hipMemcpyDeviceToDevice, st));
  }
}

void DeviceComm::alltoallv(uint64_t in, uint64_t out, uint64_t out_bytes, const std::vector<uint64_t>& soff,
                           const std::vector<uint64_t>& doff, const std::vector<uint64_t>& len, uint64_t grid_bytes,
                           uint64_t stream, int max_blocks) {
  if ((int)soff.size() != size_ || (int)doff.size() != size_ || (int)len.size() != size_)
    throw std::invalid_argument("ccmpi: alltoallv needs one offset/length per rank");
  if (grid_bytes == 0) return;  // nobody sends anything: every rank sees the same
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  uint64_t total = 0;
  for (int j = 0; j < size_; ++j) {
    if ((soff[j] | doff[j] | len[j]) % 16) throw std::invalid_argument("ccmpi: alltoallv segments must be 16-B multiples");
    if (soff[j] != total) throw std::invalid_argument("ccmpi: alltoallv send segments must be packed in peer order");
    total += len[j];
  }
  if (in % 16 || out % 16) throw std::invalid_argument("ccmpi: alltoallv buffers must be 16-B aligned");
  const uint64_t rc = code_of_(out, std::max<uint64_t>(out_bytes, 16));
  if (!rc) throw std::invalid_argument("ccmpi: alltoallv needs a registered (symmetric-heap) output on every rank");
  VArgs v{};
  v.a = args_(0, rc, (char*)out, total, 0);
  v.a.in = reinterpret_cast<const char*>(in);
  for (int j = 0; j < size_; ++j) {
    v.soff[j] = soff[j];
    v.doff[j] = doff[j];
    v.len[j] = len[j];
  }
  launch_alltoallv(v, grid_(grid_bytes, max_blocks), st);
}

void DeviceComm::alltoallv_dev(uint64_t in, uint64_t counts, uint64_t out, uint64_t out_elems, uint64_t recv_counts,
                               int elem_bytes, uint64_t stream, int max_blocks) {
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (in % 16 || out % 16) throw std::invalid_argument("ccmpi: alltoallv buffers must be 16-B aligned");
  const uint64_t row_bytes = 8ull * (size_ + 1);
  if (scratch_bytes() < row_bytes) throw std::runtime_error("ccmpi: scratch too small for alltoallv counts");
  const uint64_t rc = code_of_(out, std::max<uint64_t>(out_elems * elem_bytes, 16));
  if (!rc) throw std::invalid_argument("ccmpi: alltoallv needs a registered (symmetric-heap) output on every rank");
  // stage the counts at the start of scratch (stream-ordered before the kernel; the
  // previous collective that used scratch passed its final barrier on every rank)
  char* row = reinterpret_cast<char*>(scratch_ptr());
  CCMPI_HIP_CHECK(hipMemcpyAsync(row, (void*)counts, 8ull * size_, hipMemcpyDeviceToDevice, st));
  VDevArgs v{};
  v.a = args_(addr_code(0, 0), rc, (char*)out, 0, 0);
  v.a.in = reinterpret_cast<const char*>(in);
  v.recv_counts = reinterpret_cast<int64_t*>(recv_counts);
  v.es = (uint32_t)elem_bytes;
  v.cap = (int64_t)out_elems;
  launch_alltoallv_dev(v, std::max(1, std::min(max_blocks > 0 ? max_blocks : 256, kMaxBlocks)), st);
}

void DeviceComm::bcast(uint64_t buf, uint64_t nbytes, int root, uint64_t stream, int max_blocks, bool symmetric,
                       int mode) {
  DynScope dyn_scope(this, symmetric);
  if (nbytes == 0 || size_ == 1) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  if (symmetric && buf % 16 == 0) {
    uint64_t sc = code_of_(buf, nbytes);
    if (!sc) throw std::invalid_argument("ccmpi: symmetric bcast needs an aligned registered buffer");
    if (mode == A2A_PUSH) {
      CollArgs a = args_(0, sc, (char*)buf, nbytes, root);  // every rank publishes its buffer as the result
      a.in = reinterpret_cast<const char*>(buf);
      launch_move(MOVE_BCAST_PUSH, a, size_, grid_(nbytes, max_blocks), st);
      return;
    }
    launch_move(MOVE_BCAST, args_(sc, 0, (char*)buf, nbytes, root), size_, grid_(nbytes, max_blocks), st);
    return;
  }
  uint64_t chunk = (scratch_bytes() / 2) / 16 * 16;
  char* stage = reinterpret_cast<char*>(scratch_ptr());
  for (uint64_t off = 0; off < nbytes; off += chunk) {
    const uint64_t n = std::min(chunk, nbytes - off);
    uint64_t sc = code_of_(buf + off, n);
    if (!sc || rank_ == root) {
      if (rank_ == root) CCMPI_HIP_CHECK(hipMemcpyAsync(stage, (void*)(buf + off), n, hipMemcpyDeviceToDevice, st));
      sc = addr_code(0, 0);
    }
    const bool out_ok = (buf + off) % 16 == 0;
    char* dst = out_ok ? (char*)(buf + off) : stage + chunk;
    launch_move(MOVE_BCAST, args_(sc, 0, dst, n, root), size_, grid_(n, max_blocks), st);
    if (!out_ok && rank_ != root)
      CCMPI_HIP_CHECK(hipMemcpyAsync((void*)(buf + off), dst, n, hipMemcpyDeviceToDevice, st));
  }
}

void DeviceComm::allgather_lastaxis(uint64_t in, uint64_t out, uint64_t rows, uint64_t row_bytes, uint64_t stream,
                                    int max_blocks, bool symmetric) {
  DynScope dyn_scope(this, symmetric);
  if (rows == 0 || row_bytes == 0) return;
  if (row_bytes % 16 || out % 16) throw std::invalid_argument("ccmpi: last-axis all-gather needs 16-B rows/output");
  const uint64_t nbytes = rows * row_bytes;
  if (nbytes * size_ >= 0xFFFFFFF0ull) throw std::invalid_argument("ccmpi: last-axis all-gather > 4 GiB");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  uint64_t sc = code_of_(in, nbytes);
  if (!sc) {
    if (symmetric) throw std::invalid_argument("ccmpi: symmetric last-axis all-gather needs a registered input");
    if (nbytes > scratch_bytes()) throw std::runtime_error("ccmpi: last-axis all-gather input exceeds scratch");
    CCMPI_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(scratch_ptr()), (void*)in, nbytes, hipMemcpyDeviceToDevice, st));
    sc = addr_code(0, 0);
  }
  CollArgs a = args_(sc, 0, (char*)out, row_bytes, (int)rows);
  launch_lastaxis(0, a, size_, DT_F32, OP_SUM, grid_(nbytes * size_, max_blocks), st);
}

void DeviceComm::reduce_scatter_lastaxis(uint64_t in, uint64_t out, uint64_t rows, uint64_t k, int dtype, int op,
                                         uint64_t stream, int max_blocks, bool symmetric) {
  DynScope dyn_scope(this, symmetric);
  const uint64_t es = dtype_bytes(dtype), row_bytes = k * es;
  if (rows == 0 || k == 0) return;
  if (!device_reduce_supported(dtype, op)) throw std::invalid_argument("ccmpi: unsupported device reduction");
  if (row_bytes % 16 || out % 16) throw std::invalid_argument("ccmpi: last-axis reduce-scatter needs 16-B rows/output");
  const uint64_t nbytes = rows * row_bytes * size_;
  if (nbytes >= 0xFFFFFFF0ull) throw std::invalid_argument("ccmpi: last-axis reduce-scatter > 4 GiB");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = S(stream);
  uint64_t sc = code_of_(in, nbytes);
  if (!sc) {
    if (symmetric) throw std::invalid_argument("ccmpi: symmetric last-axis reduce-scatter needs a registered input");
    if (nbytes > scratch_bytes()) throw std::runtime_error("ccmpi: last-axis reduce-scatter input exceeds scratch");
    CCMPI_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(scratch_ptr()), (void*)in, nbytes, hipMemcpyDeviceToDevice, st));
    sc = addr_code(0, 0);
  }
  CollArgs a = args_(sc, 0, (char*)out, row_bytes, (int)rows);
  launch_lastaxis(1, a, size_, dtype, op, grid_(rows * row_bytes, max_blocks), st);
}

void DeviceComm::local_reduce(const std::vector<uint64_t>& ins, uint64_t out, uint64_t count, int dtype, int op,
                              uint64_t stream) {
  if (ins.empty() || ins.size() > (size_t)kMaxRanks) throw std::invalid_argument("ccmpi: local_reduce takes 1..16 inputs");
  LocalReduceArgs a{};
  for (size_t i = 0; i < ins.size(); ++i) {
    if (ins[i] % 16) throw std::invalid_argument("ccmpi: local_reduce inputs must be 16-B aligned");
    a.in[i] = reinterpret_cast<const char*>(ins[i]);
  }
  if (out % 16) throw std::invalid_argument("ccmpi: local_reduce output must be 16-B aligned");
  a.n_in = (int)ins.size();
  a.out = reinterpret_cast<char*>(out);
  a.nbytes = count * dtype_bytes(dtype);
  if (!a.nbytes) return;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  launch_local_reduce(a, dtype, op, S(stream));
}

// ---------------------------------------------------------------------------
// RCCL
// ---------------------------------------------------------------------------
std::string DeviceComm::rccl_unique_id() {
  ncclUniqueId id;
  CCMPI_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

void DeviceComm::rccl_init(const std::string& uid) {
  if (nccl_) return;
  if (uid.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("ccmpi: bad RCCL unique id");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  CCMPI_NCCL_CHECK(ncclCommInitRank(&nccl_, size_, id, rank_));
}

int DeviceComm::rccl_register_segments() {
  if (!nccl_) return 0;
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  for (size_t s = rccl_regs_.size(); s < segs_.size(); ++s) {
    void* h = nullptr;
    if (ncclCommRegister(nccl_, segs_[s].local, segs_[s].bytes, &h) != ncclSuccess) h = nullptr;  // best effort
    rccl_regs_.push_back(h);
  }
  int n = 0;
  for (void* h : rccl_regs_) n += h != nullptr;
  return n;
}

uint64_t DeviceComm::staging_chunk_(uint64_t budget, uint64_t align) const {
  uint64_t c = budget;
  if (chunk_cap_ && chunk_cap_ < c) c = chunk_cap_;
  return c / align * align;
}

void DeviceComm::rccl_split_from(DeviceComm* parent, int color, int key) {
  if (!parent || !parent->nccl_) throw std::runtime_error("ccmpi: parent has no RCCL communicator to split");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  ncclComm_t child = nullptr;
  CCMPI_NCCL_CHECK(ncclCommSplit(parent->nccl_, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &child, nullptr));
  if (color >= 0) nccl_ = child;
}

void DeviceComm::rccl_split_leave(DeviceComm* parent) {
  if (!parent || !parent->nccl_) throw std::runtime_error("ccmpi: parent has no RCCL communicator to split");
  CCMPI_HIP_CHECK(hipSetDevice(parent->device_));
  ncclComm_t none = nullptr;
  CCMPI_NCCL_CHECK(ncclCommSplit(parent->nccl_, NCCL_SPLIT_NOCOLOR, 0, &none, nullptr));
}

#define CCMPI_NEED_RCCL() \
  if (!nccl_) throw std::runtime_error("ccmpi: RCCL communicator not initialised")

void DeviceComm::rccl_allreduce(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, uint64_t stream) {
  CCMPI_NEED_RCCL();
  CCMPI_NCCL_CHECK(ncclAllReduce((void*)in, (void*)out, count, nccl_dt(dtype), nccl_op(op), nccl_, S(stream)));
}

void DeviceComm::rccl_reduce_scatter(uint64_t in, uint64_t out, uint64_t count, int dtype, int op, uint64_t stream) {
  CCMPI_NEED_RCCL();
  CCMPI_NCCL_CHECK(ncclReduceScatter((void*)in, (void*)out, count, nccl_dt(dtype), nccl_op(op), nccl_, S(stream)));
}

void DeviceComm::rccl_allgather(uint64_t in, uint64_t out, uint64_t count, int dtype, uint64_t stream) {
  CCMPI_NEED_RCCL();
  CCMPI_NCCL_CHECK(ncclAllGather((void*)in, (void*)out, count, nccl_dt(dtype), nccl_, S(stream)));
}

void DeviceComm::rccl_alltoall(uint64_t in, uint64_t out, uint64_t count, int dtype, uint64_t stream) {
  CCMPI_NEED_RCCL();
  CCMPI_NCCL_CHECK(ncclAllToAll((void*)in, (void*)out, count, nccl_dt(dtype), nccl_, S(stream)));
}

void DeviceComm::rccl_bcast(uint64_t buf, uint64_t count, int dtype, int root, uint64_t stream) {
  CCMPI_NEED_RCCL();
  CCMPI_NCCL_CHECK(ncclBroadcast((void*)buf, (void*)buf, count, nccl_dt(dtype), root, nccl_, S(stream)));
}

void DeviceComm::p2p_pairwise_alltoall(uint64_t in, uint64_t out, uint64_t bytes_per_peer, uint64_t stream) {
  CCMPI_NEED_RCCL();
  hipStream_t st = S(stream);
  char* i = reinterpret_cast<char*>(in);
  char* o = reinterpret_cast<char*>(out);
  CCMPI_HIP_CHECK(hipMemcpyAsync(o + rank_ * bytes_per_peer, i + rank_ * bytes_per_peer, bytes_per_peer,
                                 hipMemcpyDeviceToDevice, st));
  // reference myAlltoall2 (mpi_wrapper/comm.py:162-199): pairwise rounds; round k
  // exchanges with rank+k / rank-k, each round one grouped send+recv.
  for (int k = 1; k < size_; ++k) {
    int to = (rank_ + k) % size_, from = (rank_ - k + size_) % size_;
    CCMPI_NCCL_CHECK(ncclGroupStart());
    CCMPI_NCCL_CHECK(ncclSend(i + to * bytes_per_peer, bytes_per_peer, ncclUint8, to, nccl_, st));
    CCMPI_NCCL_CHECK(ncclRecv(o + from * bytes_per_peer, bytes_per_peer, ncclUint8, from, nccl_, st));
    CCMPI_NCCL_CHECK(ncclGroupEnd());
  }
}

std::string DeviceComm::fused_alloc() {
  if (fused_state_) throw std::runtime_error("ccmpi: fused GEMM state already allocated");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  CCMPI_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fused_state_), sizeof(gemm::FusedState),
                                        hipDeviceMallocUncached));
  CCMPI_HIP_CHECK(hipMemset(fused_state_, 0, sizeof(gemm::FusedState)));
  CCMPI_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&fused_tab_dev_), sizeof(gemm::FusedTable)));
  CCMPI_HIP_CHECK(hipDeviceSynchronize());
  hipIpcMemHandle_t h;
  CCMPI_HIP_CHECK(hipIpcGetMemHandle(&h, fused_state_));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void DeviceComm::fused_connect(const std::vector<std::string>& handles) {
  if (!fused_state_ || (int)handles.size() != size_)
    throw std::invalid_argument("ccmpi: fused_connect needs fused_alloc and one handle per rank");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  for (int j = 0; j < size_; ++j) {
    if (j == rank_) {
      fused_tab_.state[j] = fused_state_;
      continue;
    }
    fused_tab_.state[j] = static_cast<gemm::FusedState*>(ipc_open(handles[j]));
    opened_.push_back(handles[j]);
  }
  CCMPI_HIP_CHECK(hipMemcpy(fused_tab_dev_, &fused_tab_, sizeof(fused_tab_), hipMemcpyHostToDevice));
}

void DeviceComm::set_fused_inbox(uint64_t ptr, uint64_t bytes, const std::vector<uint64_t>& codes) {
  if (!fused_tab_dev_ || (int)codes.size() != size_) throw std::invalid_argument("ccmpi: set_fused_inbox before fused_connect");
  if (ptr % 16 || find(ptr, bytes, nullptr) <= 0 || codes[rank_] != code_of_(ptr, bytes))
    throw std::invalid_argument("ccmpi: the fused inbox must be an aligned symmetric allocation");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  CCMPI_HIP_CHECK(hipDeviceSynchronize());  // no fused GEMM in flight reads the old table
  for (int j = 0; j < size_; ++j) fused_tab_.inbox_code[j] = codes[j];
  CCMPI_HIP_CHECK(hipMemcpy(fused_tab_dev_, &fused_tab_, sizeof(fused_tab_), hipMemcpyHostToDevice));
  fused_inbox_bytes_ = bytes;
}

void DeviceComm::gemm_rowpar(uint64_t A, uint64_t B, uint64_t out, uint64_t bias, int M, int N, int K, int lda,
                             int ldb, int ldc, float alpha, int bias_kind, uint64_t stream) {
  if (M <= 0 || N <= 0) return;
  if (!fused_ready()) throw std::runtime_error("ccmpi: fused row-parallel GEMM not set up");
  const int tiles = gemm::gemm_w4_tiles(M, N);
  const uint64_t need = (uint64_t)((tiles + size_ - 1) / size_) * size_ * gemm::kFusedTileBytes;
  if (tiles > gemm::kFusedMaxTiles || need > fused_inbox_bytes_)
    throw std::invalid_argument("ccmpi: fused row-parallel GEMM: output too large for the inbox / tile table");
  if (K % 64 || lda % 8 || ldb % 8 || ldc % 8 || N % 8 || (A % 16) || (B % 16) || (out % 16) ||
      (uint64_t)M * ldc * 2 >= 0x7ffffff0ull)
    throw std::invalid_argument("ccmpi: fused row-parallel GEMM needs K % 64 == 0, 16-B aligned rows, N % 8 == 0");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  uint64_t oc = 0;
  {
    DynScope dyn_scope(this, true);  // the caller registered `out` (heap block or on-demand slot)
    oc = code_of_(out, (uint64_t)M * ldc * 2);
  }
  if (!oc) throw std::invalid_argument("ccmpi: fused row-parallel GEMM: the output must be registered on every rank");
  gemm::GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B),
                   reinterpret_cast<void*>(out), reinterpret_cast<const void*>(bias), M, N, K, lda, ldb, ldc, alpha, 0,
                   bias_kind, 0, 1, 1};
  gemm::FusedArgs f{dev_pt_, fused_tab_dev_, oc, ++fused_seq_, timeout_ticks_};
  hipStream_t st = S(stream);
  gemm::launch_gemm_nt_w4_fused(g, f, st);
  CCMPI_HIP_CHECK(hipGetLastError());
  gemm::launch_fused_wait(f, tiles, st);
  CCMPI_HIP_CHECK(hipGetLastError());
}

void DeviceComm::gemm_push_rowpar(uint64_t A, uint64_t B, uint64_t out, uint64_t inbox, int M, int N, int K, int lda,
                                  int ldb, float alpha, uint64_t stream, int max_blocks) {
  if (M <= 0 || N <= 0) return;
  if (size_ < 2 || size_ > kMaxRanks) throw std::invalid_argument("ccmpi: push row-parallel GEMM needs 2..16 ranks");
  const int rows = M / size_;
  const uint64_t nbytes = (uint64_t)M * N * 2;
  if (rows * size_ != M || rows % 256 || N % 8 || (out % 16) || (inbox % 16) || nbytes >= 0x7ffffff0ull)
    throw std::invalid_argument("ccmpi: push row-parallel GEMM needs M % (256 p) == 0, N % 8 == 0, 16-B aligned buffers");
  gemm::GemmArgs g{reinterpret_cast<const uint16_t*>(A), reinterpret_cast<const uint16_t*>(B), nullptr, nullptr, M, N, K,
                   lda, ldb, N, alpha, 0, 0, 0, 1, 1};
  if (!gemm::gemm_ring_ok(g, 0, 0)) throw std::invalid_argument("ccmpi: push row-parallel GEMM: K % 64 == 0, 16-B rows");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  const std::vector<uint64_t> tgt = push_targets(inbox, nbytes);
  uint16_t* push[kMaxRanks] = {};
  for (int j = 0; j < size_; ++j) push[j] = reinterpret_cast<uint16_t*>(tgt[j]);
  g.C = push[rank_];
  hipStream_t st = S(stream);
  gemm::launch_gemm_ring(g, 0, 0, st, nullptr, 0, push, rows);
  CCMPI_HIP_CHECK(hipGetLastError());
  inbox_to_local(inbox, out, nbytes, DT_BF16, stream, max_blocks);
}

std::vector<uint64_t> DeviceComm::push_targets(uint64_t inbox, uint64_t nbytes) {
  if (size_ < 2 || nbytes % (16ull * size_) || inbox % 16)
    throw std::invalid_argument("ccmpi: push inbox needs >= 2 ranks, nbytes % (16 p) == 0, a 16-B aligned block");
  uint64_t ic = 0;
  {
    DynScope dyn_scope(this, true);
    ic = code_of_(inbox, nbytes);
  }
  if (!ic) throw std::invalid_argument("ccmpi: push inbox must be a symmetric heap block");
  // block j of this rank's partial -> rank j's inbox, slot [rank_] (peer-mapped address)
  const int s = (int)(ic >> 56) - 1;
  const uint64_t off = ic & ((1ull << 56) - 1), shard = nbytes / size_;
  std::vector<uint64_t> out(size_);
  for (int j = 0; j < size_; ++j) {
    char* base = host_pt_.seg[j][s];
    if (!base) throw std::runtime_error("ccmpi: push inbox: peer segment not mapped");
    out[j] = reinterpret_cast<uint64_t>(base + off + (uint64_t)rank_ * shard);
  }
  return out;
}

void DeviceComm::inbox_to_local(uint64_t inbox, uint64_t out, uint64_t nbytes, int dtype, uint64_t stream,
                                int max_blocks) {
  if (size_ < 2 || nbytes % (16ull * size_) || inbox % 16 || out % 16 || nbytes >= 0x7ffffff0ull)
    throw std::invalid_argument("ccmpi: inbox_to_local needs >= 2 ranks, nbytes % (16 p) == 0, 16-B aligned buffers");
  if (dtype != DT_BF16 && dtype != DT_F32) throw std::invalid_argument("ccmpi: inbox_to_local sums bf16 / fp32");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  uint64_t ic = 0;
  {
    DynScope dyn_scope(this, true);
    ic = code_of_(inbox, nbytes);
  }
  if (!ic) throw std::invalid_argument("ccmpi: inbox_to_local: the inbox must be a symmetric heap block");
  launch_inbox_to_local(args_(ic, 0, reinterpret_cast<char*>(out), nbytes, 0), size_, dtype,
                        grid_(nbytes / size_, max_blocks), S(stream));
}

void DeviceComm::inbox_mean(uint64_t inbox, uint64_t out, uint64_t nbytes, int rows, uint64_t stream, int max_blocks) {
  // nbytes: the whole fp32 z (rows of 16 floats); every owner's block holds whole sequences
  const uint64_t shard = nbytes / (size_ > 0 ? size_ : 1);
  if (size_ < 2 || rows < 1 || nbytes % (64ull * rows * size_) || inbox % 16 || out % 16 || nbytes >= 0x7ffffff0ull)
    throw std::invalid_argument("ccmpi: inbox_mean needs >= 2 ranks, whole sequences (rows x 16 fp32) per rank, "
                                "16-B aligned buffers");
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  uint64_t ic = 0, oc = 0;
  const uint64_t out_bytes = nbytes / rows;
  {
    DynScope dyn_scope(this, true);
    ic = code_of_(inbox, nbytes);
    oc = code_of_(out, out_bytes);
  }
  if (!ic || !oc) throw std::invalid_argument("ccmpi: inbox_mean: the inbox and the output must be symmetric heap blocks");
  const uint64_t groups = shard / (64ull * rows);
  const int grid = std::max(1, std::min<int>((int)((groups * 4 + 255) / 256), max_blocks > 0 ? max_blocks : 64));
  launch_inbox_mean(args_(ic, oc, reinterpret_cast<char*>(out), nbytes, rows), size_, grid, S(stream));
}

uint32_t DeviceComm::error_code() {
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  CCMPI_HIP_CHECK(hipDeviceSynchronize());
  uint32_t e = 0;
  CCMPI_HIP_CHECK(hipMemcpy(&e, &sig_->error, sizeof(e), hipMemcpyDeviceToHost));
  return e;
}

void DeviceComm::set_inbox(uint64_t ptr, uint64_t bytes) {
  if (ptr && (ptr % 16 || find(ptr, bytes, nullptr) <= 0))
    throw std::invalid_argument("ccmpi: the push inbox must be an aligned symmetric allocation");
  inbox_ptr_ = ptr;
  inbox_bytes_ = bytes;
}

void DeviceComm::reset_state() {
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  CCMPI_HIP_CHECK(hipDeviceSynchronize());
  CCMPI_HIP_CHECK(hipMemset(sig_, 0, sizeof(Signals)));
  CCMPI_HIP_CHECK(hipMemset(epochs_, 0, sizeof(uint64_t) * kMaxBlocks));
  CCMPI_HIP_CHECK(hipMemset(ll_state_, 0, 2 * sizeof(uint32_t)));
  if (ll_buf_) CCMPI_HIP_CHECK(hipMemset(ll_buf_, 0, 2ull * size_ * 2 * ll_max_));
  if (fused_state_) CCMPI_HIP_CHECK(hipMemset(fused_state_, 0, sizeof(gemm::FusedState)));
  fused_seq_ = 0;
  CCMPI_HIP_CHECK(hipDeviceSynchronize());
  __atomic_store_n(host_err_, 0u, __ATOMIC_RELEASE);
}

uint32_t DeviceComm::poll_error() const {
  return __atomic_load_n(host_err_, __ATOMIC_ACQUIRE);
}

void DeviceComm::clear_error() {
  __atomic_store_n(host_err_, 0u, __ATOMIC_RELEASE);
  CCMPI_HIP_CHECK(hipSetDevice(device_));
  CCMPI_HIP_CHECK(hipMemset(&sig_->error, 0, sizeof(uint32_t)));
}

}  // namespace dev
}  // namespace ccmpi
