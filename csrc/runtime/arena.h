// HBM budget arena + parameter-cache bookkeeping for the MI355X executor.
//
// The reference has no memory manager: a "node" is a float that goes up and down
// (/root/reference/schedulers.py:86-95,125-126). Here each GPU owns ONE slab carved
// from HBM (a single torch allocation of `capacity` bytes — the memory-regime cap),
// and this arena hands out offsets inside it: best-fit, coalescing, 256-byte aligned
// (keeps every tensor 16-B aligned for dwordx4 loads and cache-line aligned for the
// kernels). Keeping the whole budget in one slab means fragmentation, peak usage and
// the cap are measured, not estimated, and the executor never calls hipMalloc on the
// hot path (hipMalloc/hipFree would also break hipGraph capture).
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace dls {

class Arena {
 public:
  explicit Arena(uint64_t capacity, uint64_t align = 256);
  // Returns the byte offset, or -1 if no free block is large enough.
  int64_t alloc(uint64_t bytes);
  // Carve exactly [off, off + bytes) out of a free block (a warm start that must keep a
  // resident block where it already is). False if that range is not entirely free.
  bool reserve(uint64_t off, uint64_t bytes);
  void release(int64_t offset);
  uint64_t capacity() const { return capacity_; }
  uint64_t used() const { return used_; }
  uint64_t peak() const { return peak_; }
  uint64_t largest_free() const;
  size_t num_free_blocks() const { return free_by_off_.size(); }
  size_t num_live() const { return live_.size(); }
  void reset_peak() { peak_ = used_; }

 private:
  void insert_free(uint64_t off, uint64_t size);
  void erase_free(std::map<uint64_t, uint64_t>::iterator it);
  uint64_t capacity_, align_, used_ = 0, peak_ = 0;
  std::map<uint64_t, uint64_t> free_by_off_;            // offset -> size
  std::multimap<uint64_t, uint64_t> free_by_size_;      // size -> offset
  std::unordered_map<uint64_t, uint64_t> live_;         // offset -> size
};

// Residency table for model parameters on one device. The executor asks
// `acquire(param, bytes)` before a node runs; a miss allocates in the arena (after
// evicting victims chosen by the caller's policy or by least-recent use) and counts a
// fill, a hit bumps recency. Counters feed the `param_loads / param_evictions` CSV
// columns (SURVEY §5 metrics row) — real fills, unlike the reference's replay which
// never models reloads.
class ParamCache {
 public:
  explicit ParamCache(Arena* arena) : arena_(arena) {}
  bool resident(const std::string& p) const { return table_.count(p) != 0; }
  int64_t offset(const std::string& p) const;
  // Returns {offset, was_hit}. offset -1 => could not make room.
  std::pair<int64_t, bool> acquire(const std::string& p, uint64_t bytes, bool allow_evict = true);
  bool evict(const std::string& p);
  void pin(const std::string& p, bool pinned);
  std::vector<std::string> residents() const;
  uint64_t hits() const { return hits_; }
  uint64_t misses() const { return misses_; }
  uint64_t evictions() const { return evictions_; }
  uint64_t reloads() const { return reloads_; }
  uint64_t bytes_filled() const { return bytes_filled_; }

 private:
  struct Entry {
    int64_t off;
    uint64_t bytes;
    uint64_t last_use;
    bool pinned;
  };
  Arena* arena_;
  std::unordered_map<std::string, Entry> table_;
  std::unordered_map<std::string, int> ever_loaded_;
  uint64_t clock_ = 0, hits_ = 0, misses_ = 0, evictions_ = 0, reloads_ = 0, bytes_filled_ = 0;
};

}  // namespace dls
