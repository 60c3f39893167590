#include "arena.h"

#include <algorithm>
#include <stdexcept>

namespace dls {

Arena::Arena(uint64_t capacity, uint64_t align) : capacity_(capacity), align_(align ? align : 1) {
  if ((align_ & (align_ - 1)) != 0) throw std::invalid_argument("alignment must be a power of two");
  if (capacity_ > 0) insert_free(0, capacity_);
}

void Arena::insert_free(uint64_t off, uint64_t size) {
  free_by_off_.emplace(off, size);
  free_by_size_.emplace(size, off);
}

void Arena::erase_free(std::map<uint64_t, uint64_t>::iterator it) {
  auto range = free_by_size_.equal_range(it->second);
  for (auto s = range.first; s != range.second; ++s) {
    if (s->second == it->first) {
      free_by_size_.erase(s);
      break;
    }
  }
  free_by_off_.erase(it);
}

int64_t Arena::alloc(uint64_t bytes) {
  if (bytes == 0) bytes = 1;
  const uint64_t need = (bytes + align_ - 1) & ~(align_ - 1);
  auto it = free_by_size_.lower_bound(need);  // best fit: smallest block >= need
  if (it == free_by_size_.end()) return -1;
  const uint64_t off = it->second, size = it->first;
  erase_free(free_by_off_.find(off));
  if (size > need) insert_free(off + need, size - need);
  live_.emplace(off, need);
  used_ += need;
  peak_ = std::max(peak_, used_);
  return static_cast<int64_t>(off);
}

bool Arena::reserve(uint64_t off, uint64_t bytes) {
  if (bytes == 0) bytes = 1;
  const uint64_t need = (bytes + align_ - 1) & ~(align_ - 1);
  if (off % align_ != 0) return false;
  // the free block that contains [off, off + need)
  auto it = free_by_off_.upper_bound(off);
  if (it == free_by_off_.begin()) return false;
  --it;
  const uint64_t boff = it->first, bsize = it->second;
  if (off < boff || off + need > boff + bsize) return false;
  erase_free(it);
  if (off > boff) insert_free(boff, off - boff);
  if (off + need < boff + bsize) insert_free(off + need, boff + bsize - off - need);
  live_.emplace(off, need);
  used_ += need;
  peak_ = std::max(peak_, used_);
  return true;
}

void Arena::release(int64_t offset) {
  auto lv = live_.find(static_cast<uint64_t>(offset));
  if (lv == live_.end()) throw std::invalid_argument("arena: release of unknown offset");
  uint64_t off = lv->first, size = lv->second;
  live_.erase(lv);
  used_ -= size;
  // coalesce with the right neighbour
  auto right = free_by_off_.find(off + size);
  if (right != free_by_off_.end()) {
    size += right->second;
    erase_free(right);
  }
  // coalesce with the left neighbour
  auto left = free_by_off_.lower_bound(off);
  if (left != free_by_off_.begin()) {
    --left;
    if (left->first + left->second == off) {
      off = left->first;
      size += left->second;
      erase_free(left);
    }
  }
  insert_free(off, size);
}

uint64_t Arena::largest_free() const { return free_by_size_.empty() ? 0 : free_by_size_.rbegin()->first; }

int64_t ParamCache::offset(const std::string& p) const {
  auto it = table_.find(p);
  return it == table_.end() ? -1 : it->second.off;
}

std::pair<int64_t, bool> ParamCache::acquire(const std::string& p, uint64_t bytes, bool allow_evict) {
  ++clock_;
  auto it = table_.find(p);
  if (it != table_.end()) {
    it->second.last_use = clock_;
    ++hits_;
    return {it->second.off, true};
  }
  int64_t off = arena_->alloc(bytes);
  while (off < 0 && allow_evict) {
    // least-recently-used unpinned victim
    auto victim = table_.end();
    for (auto e = table_.begin(); e != table_.end(); ++e) {
      if (e->second.pinned) continue;
      if (victim == table_.end() || e->second.last_use < victim->second.last_use) victim = e;
    }
    if (victim == table_.end()) break;
    arena_->release(victim->second.off);
    table_.erase(victim);
    ++evictions_;
    off = arena_->alloc(bytes);
  }
  if (off < 0) return {-1, false};
  table_.emplace(p, Entry{off, bytes, clock_, false});
  ++misses_;
  bytes_filled_ += bytes;
  if (ever_loaded_[p]++ > 0) ++reloads_;
  return {off, false};
}

bool ParamCache::evict(const std::string& p) {
  auto it = table_.find(p);
  if (it == table_.end()) return false;
  arena_->release(it->second.off);
  table_.erase(it);
  ++evictions_;
  return true;
}

void ParamCache::pin(const std::string& p, bool pinned) {
  auto it = table_.find(p);
  if (it != table_.end()) it->second.pinned = pinned;
}

std::vector<std::string> ParamCache::residents() const {
  std::vector<std::string> out;
  out.reserve(table_.size());
  for (const auto& kv : table_) out.push_back(kv.first);
  std::sort(out.begin(), out.end());
  return out;
}

}  // namespace dls
