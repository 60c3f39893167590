// Host-side pieces of the executor's point-to-point path that carry no GPU or torch types, so
// they compile into the pybind op library AND into the sanitizer selftest (csrc/tests/
// core_selftest.cpp, ASan/UBSan and TSan with one thread per rank):
//
//  * P2PMatcher — pairing of posted sends and receives with ncclSend / ncclRecv semantics: FIFO
//    per (src, dst) pair, a post that finds its counterpart pending is matched on the spot (the
//    caller's on_match runs under the lock, e.g. to enqueue the copy), and wait() blocks until an
//    op is matched. The single-GPU loopback hub (csrc/kernels/loopback.cpp) is built on it.
//  * run_actions — the native step runner's action loop (csrc/kernels/runner.cpp): one recorded
//    steady-state step replayed against a backend — device work, events, p2p posts / waits,
//    coalesced groups, and the end-of-step drain of every p2p op still outstanding.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace dls {

template <class Op>
class P2PMatcher {
 public:
  using MatchFn = std::function<void(Op& send, Op& recv)>;

  explicit P2PMatcher(int world) : world_(world) {}

  // post a send (self -> peer) or a receive (peer -> self); returns its id
  int64_t post(bool send, int self, int peer, Op op, const MatchFn& on_match) {
    if (self < 0 || self >= world_ || peer < 0 || peer >= world_ || self == peer)
      throw std::invalid_argument("p2p: bad ranks " + std::to_string(self) + " -> " + std::to_string(peer));
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t id = next_++;
    const auto key = send ? std::make_pair(self, peer) : std::make_pair(peer, self);
    auto& other = send ? recvs_[key] : sends_[key];
    Entry& e = ops_[id];
    e.op = std::move(op);
    e.send = send;
    e.self = self;
    e.peer = peer;
    if (!other.empty()) {
      const int64_t oid = other.front();
      other.pop_front();
      Entry& o = ops_.at(oid);
      Entry& s = send ? e : o;
      Entry& r = send ? o : e;
      try {
        on_match(s.op, r.op);  // may throw (size mismatch)
      } catch (const std::exception& ex) {
        // both ends fail with the real error: the counterpart was already taken off its FIFO,
        // so its wait() must not run into the timeout and report "never matched". The posting
        // op's own entry is dropped here: its id is never returned, so nobody could wait() it
        // (it would stay outstanding for the hub's lifetime)
        o.error = ex.what();
        o.matched = true;
        ops_.erase(id);
        cv_.notify_all();
        throw;
      }
      e.matched = o.matched = true;
      ++matched_pairs_;
      cv_.notify_all();
    } else {
      (send ? sends_[key] : recvs_[key]).push_back(id);
    }
    return id;
  }

  // block until op ``id`` is matched; false on timeout. On success the op is handed back and
  // forgotten (each op is waited for exactly once).
  bool wait(int64_t id, double timeout_s, Op* out = nullptr) {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = ops_.find(id);
    if (it == ops_.end()) throw std::invalid_argument("p2p: unknown or already waited op " + std::to_string(id));
    // system_clock deadline: libstdc++ turns a steady_clock wait into pthread_cond_clockwait,
    // which this toolchain's ThreadSanitizer does not intercept (it then reports the mutex the
    // wait released as locked twice); timedwait is intercepted
    const auto deadline = std::chrono::system_clock::now() +
                          std::chrono::duration_cast<std::chrono::system_clock::duration>(
                              std::chrono::duration<double>(timeout_s));
    if (!cv_.wait_until(lk, deadline, [&] { return ops_.at(id).matched; })) return false;
    if (!ops_.at(id).error.empty()) {
      const std::string err = ops_.at(id).error;
      ops_.erase(id);
      throw std::runtime_error("p2p: " + err);
    }
    if (out) *out = std::move(ops_.at(id).op);
    ops_.erase(id);
    return true;
  }

  // the (self, peer, is_send) of an op not yet waited for
  bool describe(int64_t id, int* self, int* peer, bool* send) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = ops_.find(id);
    if (it == ops_.end()) return false;
    *self = it->second.self;
    *peer = it->second.peer;
    *send = it->second.send;
    return true;
  }

  int64_t outstanding() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int64_t)ops_.size();
  }
  int64_t matched_pairs() {
    std::lock_guard<std::mutex> lk(mu_);
    return matched_pairs_;
  }
  int world() const { return world_; }

 private:
  struct Entry {
    Op op{};
    bool send = false, matched = false;
    int self = 0, peer = 0;
    std::string error;  // set on both ends when the match itself failed (on_match threw)
  };
  int world_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::pair<int, int>, std::deque<int64_t>> sends_, recvs_;  // unmatched, by (src, dst)
  std::unordered_map<int64_t, Entry> ops_;
  int64_t next_ = 0;
  int64_t matched_pairs_ = 0;
};

// ------------------------------------------------------------------ step runner action loop

enum ActKind : int { GRAPH = 0, PULL, MEMCPY, MEMSET, EV_RECORD, EV_WAIT, SEND, RECV, WORK_WAIT, PYCALL, GROUP_BEGIN,
                     GROUP_END };

// One recorded action. ``Tensor`` / ``Fn`` are the backend's buffer and callback types.
template <class Tensor, class Fn>
struct StepAction {
  ActKind kind;
  int stream = 0;  // 0 compute, 1 copy stream
  uint64_t exec = 0;
  void* dst = nullptr;
  const void* src = nullptr;
  size_t bytes = 0;
  int blocks = 0;
  int value = 0;  // SEND / RECV: work index; GROUP_END: one past the group's last work index
  int index = 0;  // event index / work index / peer rank / GROUP_END: the group's first work index
  Tensor tensor{};
  Fn fn{};
};

// Replay ``acts`` (whose p2p ops carry work indices 0..n_works-1) against backend ``b``:
//   b.graph(a) b.pull(a) b.memcpy(a) b.memset(a) b.record(a) b.wait_event(a) b.pycall(a)
//   b.post(a) -> Work          (SEND / RECV)
//   b.group_begin() -> bool    (true: the backend coalesces the group into one work)
//   b.group_end() -> Work      (the coalesced group's work)
//   b.wait(Work&)              (and Work is default-constructible, testable with bool(w))
// Every p2p op still outstanding when the step ends is waited for, as the Python step does.
template <class Backend, class Action>
void run_actions(const std::vector<Action>& acts, int n_works, Backend& b) {
  using Work = typename Backend::Work;
  std::vector<Work> works(n_works);
  bool coalescing = false;
  for (const auto& a : acts) {
    switch (a.kind) {
      case GRAPH: b.graph(a); break;
      case PULL: b.pull(a); break;
      case MEMCPY: b.memcpy(a); break;
      case MEMSET: b.memset(a); break;
      case EV_RECORD: b.record(a); break;
      case EV_WAIT: b.wait_event(a); break;
      case PYCALL: b.pycall(a); break;
      case SEND:
      case RECV:
        works.at(a.value) = b.post(a);
        break;
      case GROUP_BEGIN:
        coalescing = b.group_begin();
        break;
      case GROUP_END:
        if (coalescing) {  // ONE work for the whole group: every op of it waits on it
          Work w = b.group_end();
          for (int i = a.index; i < a.value; ++i) works.at(i) = w;
          coalescing = false;
        }
        break;
      case WORK_WAIT: {
        Work& w = works.at(a.index);
        if (w) {
          b.wait(w);
          w = Work{};
        }
        break;
      }
    }
  }
  for (auto& w : works)
    if (w) b.wait(w);
}

}  // namespace dls
