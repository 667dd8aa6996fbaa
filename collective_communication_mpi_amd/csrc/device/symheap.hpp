// Symmetric heap: a best-fit allocator with coalescing over IPC-registered
// arenas (symmetric segments).  Every rank runs the same allocation / free
// sequence (SPMD), so equal requests land at equal offsets; the collectives do
// not depend on that (every kernel publishes its buffers' addresses), it only
// keeps the arenas' growth in lockstep.  Blocks are handed to Python as
// DLPack capsules whose deleter returns the block when the last view of the
// tensor dies, like torch's caching allocator (stream order: a freed block is
// reused by later work on the same stream only).
#pragma once

#include <stdint.h>

#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace ccmpi {
namespace dev {

class SymHeap : public std::enable_shared_from_this<SymHeap> {
 public:
  static constexpr uint64_t kAlign = 256;

  // Register a fresh arena (an already IPC-registered range).
  void add_arena(uint64_t base, uint64_t bytes);
  // Best-fit; 0 when no arena has room (the caller grows the heap collectively).
  uint64_t alloc(uint64_t bytes);
  void release(uint64_t ptr);
  uint64_t used_bytes() const;
  uint64_t capacity() const;
  uint64_t largest_free() const;
  int live_blocks() const;

 private:
  mutable std::mutex mu_;
  std::map<uint64_t, uint64_t> free_;   // address -> length (coalesced)
  std::map<uint64_t, uint64_t> live_;   // address -> length
  std::vector<std::pair<uint64_t, uint64_t>> arenas_;
  uint64_t used_ = 0, cap_ = 0;
};

}  // namespace dev
}  // namespace ccmpi
