// Symmetric heap allocator (see symheap.hpp).
#include "symheap.hpp"

#include <algorithm>
#include <stdexcept>

namespace ccmpi {
namespace dev {

void SymHeap::add_arena(uint64_t base, uint64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  const uint64_t lo = (base + kAlign - 1) / kAlign * kAlign;
  if (lo >= base + bytes) throw std::invalid_argument("symheap: arena too small");
  const uint64_t len = (base + bytes - lo) / kAlign * kAlign;
  arenas_.push_back({lo, len});
  free_[lo] = len;  // arenas are distinct allocations: never coalesce across them
  cap_ += len;
}

uint64_t SymHeap::alloc(uint64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  const uint64_t need = std::max<uint64_t>(kAlign, (bytes + kAlign - 1) / kAlign * kAlign);
  auto best = free_.end();
  for (auto it = free_.begin(); it != free_.end(); ++it)  // best fit, lowest address on ties
    if (it->second >= need && (best == free_.end() || it->second < best->second)) best = it;
  if (best == free_.end()) return 0;
  const uint64_t addr = best->first, len = best->second;
  free_.erase(best);
  if (len > need) free_[addr + need] = len - need;
  live_[addr] = need;
  used_ += need;
  return addr;
}

void SymHeap::release(uint64_t ptr) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = live_.find(ptr);
  if (it == live_.end()) return;  // not ours (or already released)
  uint64_t addr = it->first, len = it->second;
  live_.erase(it);
  used_ -= len;
  auto in_same_arena = [&](uint64_t a, uint64_t b) {
    for (auto& ar : arenas_)
      if (a >= ar.first && a < ar.first + ar.second) return b >= ar.first && b < ar.first + ar.second;
    return false;
  };
  // coalesce with the following and the preceding free block of the same arena
  auto nx = free_.lower_bound(addr);
  if (nx != free_.end() && nx->first == addr + len && in_same_arena(addr, nx->first)) {
    len += nx->second;
    free_.erase(nx);
  }
  auto pv = free_.lower_bound(addr);
  if (pv != free_.begin()) {
    --pv;
    if (pv->first + pv->second == addr && in_same_arena(pv->first, addr)) {
      addr = pv->first;
      len += pv->second;
      free_.erase(pv);
    }
  }
  free_[addr] = len;
}

uint64_t SymHeap::used_bytes() const {
  std::lock_guard<std::mutex> g(mu_);
  return used_;
}

uint64_t SymHeap::capacity() const {
  std::lock_guard<std::mutex> g(mu_);
  return cap_;
}

uint64_t SymHeap::largest_free() const {
  std::lock_guard<std::mutex> g(mu_);
  uint64_t m = 0;
  for (auto& f : free_) m = std::max(m, f.second);
  return m;
}

int SymHeap::live_blocks() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int)live_.size();
}

}  // namespace dev
}  // namespace ccmpi
