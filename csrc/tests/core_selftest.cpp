// Native selftest of the scheduling core and the HBM arena, built with sanitizers
// (ASan + UBSan, or TSan with --threads N) by tests/test_sanitizers.py — SURVEY §5 "race
// detection / sanitizers": the Python layer never sees an out-of-bounds index or a data
// race in the core because this binary has already run the same code paths instrumented.
//
//   core_selftest [--instances N] [--threads T] [--seed S]
//
// Per random instance and policy it checks the invariants the Python property tests check
// (trace replay never over-commits memory, never runs a task before its dependencies,
// accounts every task as completed / failed / never-started), and it hammers the arena
// with random alloc/release sequences against a reference interval list.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../core/scheduler.h"
#include "../runtime/arena.h"
#include "../core/partition.h"
#include "../runtime/p2p_match.h"

namespace {

std::atomic<int> g_failures{0};

#define CHECK(cond, ...)                                 \
  do {                                                   \
    if (!(cond)) {                                       \
      std::fprintf(stderr, "CHECK failed: %s: ", #cond); \
      std::fprintf(stderr, __VA_ARGS__);                 \
      std::fprintf(stderr, "\n");                        \
      g_failures.fetch_add(1);                           \
    }                                                    \
  } while (0)

dls::Instance random_instance(std::mt19937& rng) {
  dls::Instance in;
  std::uniform_int_distribution<int> ntask(5, 120), nnode(1, 6), nparam(1, 40);
  const int T = ntask(rng), N = nnode(rng), P = nparam(rng);
  std::uniform_real_distribution<double> mem(0.05, 0.6), comp(0.01, 0.2), u(0.0, 1.0);
  for (int p = 0; p < P; ++p) {
    in.param_names.push_back("p" + std::to_string(p));
    in.param_cost.push_back(u(rng) < 0.5 ? 0.5 : 0.05 + u(rng));
  }
  for (int t = 0; t < T; ++t) {
    in.task_ids.push_back("t" + std::to_string(t));
    in.mem.push_back(mem(rng));
    in.compute.push_back(comp(rng));
    in.out_size.push_back(u(rng) * 0.01);
    std::vector<int> deps;
    const int nd = t == 0 ? 0 : std::uniform_int_distribution<int>(0, std::min(t, 3))(rng);
    std::set<int> seen;
    for (int k = 0; k < nd; ++k) {
      int d = std::uniform_int_distribution<int>(0, t - 1)(rng);
      if (seen.insert(d).second) deps.push_back(d);
    }
    if (u(rng) < 0.03) deps.push_back(-1);  // a dependency on an id that is not a task
    in.deps.push_back(deps);
    std::vector<int> ps;
    const int np = std::uniform_int_distribution<int>(0, 2)(rng);
    std::set<int> pseen;
    for (int k = 0; k < np; ++k) {
      int p = std::uniform_int_distribution<int>(0, P - 1)(rng);
      if (pseen.insert(p).second) ps.push_back(p);
    }
    in.params.push_back(ps);
  }
  double total = 0;
  for (int t = 0; t < T; ++t) total += in.mem[t];
  for (int p = 0; p < P; ++p) total += in.param_cost[p];
  const double regime = 0.2 + 0.9 * u(rng);
  for (int n = 0; n < N; ++n) {
    in.node_ids.push_back("n" + std::to_string(n));
    in.node_mem.push_back(total * regime / N + 0.7);
    in.node_speed.push_back(0.7 + 0.6 * u(rng));
  }
  return in;
}

void check_result(const dls::Instance& in, const dls::Result& r, int policy) {
  const int T = (int)in.task_ids.size(), N = (int)in.node_ids.size();
  std::vector<double> free_mem(in.node_mem);
  std::vector<std::set<int>> cached(N);
  std::vector<char> done(T, 0);
  for (const auto& e : r.events) {
    if (e.action == (int)dls::Action::LOAD) {
      CHECK(e.node >= 0 && e.node < N, "policy %d LOAD node %d", policy, e.node);
      CHECK(!cached[e.node].count(e.item), "policy %d double load", policy);
      cached[e.node].insert(e.item);
      free_mem[e.node] -= in.param_cost[e.item];
    } else if (e.action == (int)dls::Action::EVICT) {
      CHECK(cached[e.node].count(e.item), "policy %d evicting non-resident", policy);
      cached[e.node].erase(e.item);
      free_mem[e.node] += in.param_cost[e.item];
    } else if (e.action == (int)dls::Action::RUN) {
      CHECK(e.item >= 0 && e.item < T, "policy %d RUN item %d", policy, e.item);
      for (int d : in.deps[e.item]) CHECK(d < 0 || done[d], "policy %d dependency order (task %d)", policy, e.item);
      for (int p : in.params[e.item]) CHECK(cached[e.node].count(p), "policy %d param not resident", policy);
      CHECK(free_mem[e.node] - in.mem[e.item] >= -1e-9, "policy %d over-commit node %d", policy, e.node);
      done[e.item] = 1;
    }
    for (int n = 0; n < N; ++n) CHECK(free_mem[n] >= -1e-9, "policy %d negative free memory", policy);
  }
  // completed / failed are per-task flags
  CHECK((int)r.completed.size() == T && (int)r.failed.size() == T, "result flag vectors sized T");
  for (int t = 0; t < T; ++t) {
    CHECK(!(r.completed[t] && r.failed[t]), "policy %d task %d both completed and failed", policy, t);
    CHECK((bool)done[t] == (bool)r.completed[t], "policy %d task %d ran/completed mismatch", policy, t);
    CHECK(!r.completed[t] || (r.assigned_node[t] >= 0 && r.assigned_node[t] < N), "assigned node");
  }
  if (policy == (int)dls::Policy::EFT) {
    for (int t = 0; t < T; ++t)
      if (r.completed[t])
        CHECK(r.finish_time[t] >= r.start_time[t] && std::isfinite(r.finish_time[t]), "EFT timeline");
  }
  // dependency-respecting replay of the same placement stays finite and ordered
  std::vector<double> st, fi;
  dls::replay_with_deps(in, r.schedule, st, fi, true);
  for (int t = 0; t < T; ++t)
    if (r.completed[t]) CHECK(std::isfinite(fi[t]) && fi[t] >= st[t], "replay timeline task %d", t);
}

void arena_stress(std::mt19937& rng) {
  const uint64_t cap = 1 << 22;
  dls::Arena a(cap, 256);
  std::map<int64_t, uint64_t> live;  // reference: offset -> size
  std::uniform_int_distribution<int> op(0, 2);
  std::uniform_int_distribution<uint64_t> sz(1, 1 << 16);
  for (int it = 0; it < 20000; ++it) {
    if (live.empty() || op(rng) > 0) {
      const uint64_t s = sz(rng);
      const int64_t off = a.alloc(s);
      if (off < 0) continue;
      CHECK(off % 256 == 0, "arena alignment");
      CHECK((uint64_t)off + s <= cap, "arena bounds");
      auto nx = live.lower_bound(off);
      if (nx != live.end()) CHECK((uint64_t)off + s <= (uint64_t)nx->first, "arena overlap (next)");
      if (nx != live.begin()) {
        auto pv = std::prev(nx);
        CHECK((uint64_t)pv->first + pv->second <= (uint64_t)off, "arena overlap (prev)");
      }
      live[off] = (s + 255) / 256 * 256;
    } else {
      auto it2 = live.begin();
      std::advance(it2, std::uniform_int_distribution<size_t>(0, live.size() - 1)(rng));
      a.release(it2->first);
      live.erase(it2);
    }
    uint64_t used = 0;
    for (auto& kv : live) used += kv.second;
    CHECK(a.used() == used, "arena used %llu vs %llu", (unsigned long long)a.used(), (unsigned long long)used);
  }
  dls::ParamCache pc(&a);
  for (int it = 0; it < 2000; ++it) {
    const std::string p = "w" + std::to_string(std::uniform_int_distribution<int>(0, 60)(rng));
    auto r = pc.acquire(p, sz(rng) * 4);
    if (r.first >= 0) CHECK(pc.resident(p), "param cache residency");
  }
}

void worker(int id, int instances, unsigned seed) {
  std::mt19937 rng(seed + 7919u * (unsigned)id);
  for (int i = 0; i < instances; ++i) {
    dls::Instance in = random_instance(rng);
    for (int pol = 0; pol <= 4; ++pol) check_result(in, dls::run_policy(in, (dls::Policy)pol), pol);
    (void)dls::depth_from_sources(in);
    (void)dls::bottom_level(in);
  }
  arena_stress(rng);
}

}  // namespace

// ---- the step runner's action loop + the loopback pairing, one thread per rank (TSan: the
// matcher's lock / condition variable; ASan: work indices, buffers, group bookkeeping)
struct CpuWork {
  int64_t id = -1;
  explicit operator bool() const { return id >= 0; }
};
using CpuAction = dls::StepAction<std::vector<float>*, std::function<void()>>;
struct CpuOp {
  std::vector<float>* buf = nullptr;
};

struct CpuBackend {
  using Work = CpuWork;
  dls::P2PMatcher<CpuOp>* m = nullptr;
  int rank = 0;
  bool coalesce = false;
  void graph(const CpuAction&) {}
  void pull(const CpuAction&) {}
  void memcpy(const CpuAction&) {}
  void memset(const CpuAction&) {}
  void record(const CpuAction&) {}
  void wait_event(const CpuAction&) {}
  void pycall(const CpuAction& a) { a.fn(); }
  Work post(const CpuAction& a) {
    CpuOp op;
    op.buf = a.tensor;
    Work w;
    w.id = m->post(a.kind == dls::SEND, rank, a.index, op, [](CpuOp& s, CpuOp& r) {
      if (s.buf->size() != r.buf->size()) throw std::runtime_error("size mismatch");
      std::copy(s.buf->begin(), s.buf->end(), r.buf->begin());
    });
    return w;
  }
  bool group_begin() { return false; }  // one work per op (the gloo behaviour)
  Work group_end() { return Work{}; }
  void wait(Work& w) {
    if (!m->wait(w.id, 30.0)) {
      std::fprintf(stderr, "rank %d: p2p op %lld never matched\n", rank, (long long)w.id);
      g_failures.fetch_add(1);
    }
  }
};

// A pipeline of `world` ranks, `mb` micro-batches, each a vector of `n` floats: rank r receives
// micro-batch k from r-1 (rank 0 makes it), adds r+1, sends it on; the last rank checks it. Every
// rank's step is a recorded action list (grouped recv of k+1 with the send of k, waits before
// the compute callbacks) replayed `steps` times — the step runner's shape, run by run_actions.
void p2p_pipeline(int world, int mb, int n, int steps) {
  dls::P2PMatcher<CpuOp> m(world);
  std::vector<std::vector<std::vector<float>>> in(world, std::vector<std::vector<float>>(mb, std::vector<float>(n)));
  std::vector<std::vector<std::vector<float>>> out(world, std::vector<std::vector<float>>(mb, std::vector<float>(n)));
  std::vector<std::thread> ranks;
  for (int r = 0; r < world; ++r) {
    ranks.emplace_back([&, r] {
      std::vector<CpuAction> acts;
      int works = 0;
      std::vector<int> recv_w(mb, -1), send_w(mb, -1);
      auto add_p2p = [&](dls::ActKind k, std::vector<float>* b, int peer) {
        CpuAction a{k};
        a.tensor = b;
        a.index = peer;
        a.value = works;
        acts.push_back(a);
        return works++;
      };
      auto add_wait = [&](int w) {
        CpuAction a{dls::WORK_WAIT};
        a.index = w;
        acts.push_back(a);
      };
      auto step_no = std::make_shared<int>(0);
      {
        CpuAction a{dls::PYCALL};
        a.fn = [step_no] { ++*step_no; };
        acts.push_back(a);
      }
      if (r > 0) recv_w[0] = add_p2p(dls::RECV, &in[r][0], r - 1);
      for (int k = 0; k < mb; ++k) {
        if (r > 0) add_wait(recv_w[k]);
        CpuAction c{dls::PYCALL};
        c.fn = [&, r, k, step_no] {
          for (int i = 0; i < n; ++i) {
            const float base = r == 0 ? (float)(k * 1000 + i + *step_no) : in[r][k][i];
            out[r][k][i] = base + (float)(r + 1);
          }
        };
        acts.push_back(c);
        const bool grp = r + 1 < world && r > 0 && k + 1 < mb;
        if (grp) acts.push_back(CpuAction{dls::GROUP_BEGIN});
        const int g0 = works;
        if (r + 1 < world) send_w[k] = add_p2p(dls::SEND, &out[r][k], r + 1);
        if (r > 0 && k + 1 < mb) recv_w[k + 1] = add_p2p(dls::RECV, &in[r][k + 1], r - 1);
        if (grp) {
          CpuAction e{dls::GROUP_END};
          e.index = g0;
          e.value = works;
          acts.push_back(e);
        }
      }
      if (r + 1 == world) {  // the last rank checks every micro-batch of this step
        CpuAction c{dls::PYCALL};
        c.fn = [&, r, step_no] {
          for (int k = 0; k < mb; ++k)
            for (int i = 0; i < n; ++i) {
              const float want = (float)(k * 1000 + i + *step_no) + (float)(world * (world + 1) / 2);
              if (out[r][k][i] != want) {
                g_failures.fetch_add(1);
                std::fprintf(stderr, "p2p pipeline: step %d mb %d [%d] = %f, want %f\n", *step_no, k, i,
                             out[r][k][i], want);
                return;
              }
            }
        };
        acts.push_back(c);
      }
      CpuBackend b;
      b.m = &m;
      b.rank = r;
      for (int s = 0; s < steps; ++s) dls::run_actions(acts, works, b);
    });
  }
  for (auto& t : ranks) t.join();
  CHECK(m.outstanding() == 0, "p2p: %lld ops left unwaited", (long long)m.outstanding());
  CHECK(m.matched_pairs() == (int64_t)steps * mb * (world - 1), "p2p: %lld transfers", (long long)m.matched_pairs());
}

int main(int argc, char** argv) {
  int instances = 200, threads = 1;
  unsigned seed = 1;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--instances")) instances = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--threads")) threads = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--seed")) seed = (unsigned)std::atoi(argv[i + 1]);
  }
  // deep chain: the iterative depth / b-level must not recurse (reference Q7)
  {
    dls::Instance in;
    const int T = 20000;
    for (int t = 0; t < T; ++t) {
      in.task_ids.push_back("c" + std::to_string(t));
      in.mem.push_back(0.01);
      in.compute.push_back(0.01);
      in.out_size.push_back(0.0);
      in.deps.push_back(t ? std::vector<int>{t - 1} : std::vector<int>{});
      in.params.push_back({});
    }
    in.node_ids = {"n0"};
    in.node_mem = {10.0};
    in.node_speed = {1.0};
    auto r = dls::run_policy(in, dls::Policy::CRITICAL);
    int n = 0;
    for (int t = 0; t < T; ++t) n += r.completed[t] != 0;
    CHECK(n == T, "deep chain completed %d of %d", n, T);
  }
  // steady-state partition of a long capped chain over 3 nodes (csrc/core/partition.h)
  {
    dls::Instance in;
    const int T = 300;
    for (int t = 0; t < T; ++t) {
      in.task_ids.push_back("s" + std::to_string(t));
      in.mem.push_back(0.0);
      in.compute.push_back(1e-5 * (1 + t % 7));
      in.out_size.push_back(1e-3);
      in.deps.push_back(t ? std::vector<int>{t - 1} : std::vector<int>{});
      in.params.push_back({t});
      in.param_names.push_back("p" + std::to_string(t));
      in.param_cost.push_back(0.5);
      in.param_refill.push_back(0.01 * (1 + t % 3));
    }
    in.node_ids = {"n0", "n1", "n2"};
    in.node_mem = {20.0, 20.0, 20.0};
    in.node_speed = {1.0, 1.0, 1.0};
    auto part = dls::steady_partition(in);
    CHECK(part.feasible && part.stage_node.size() == 3, "partition: feasible over 3 stages");
    auto busy = dls::steady_node_cost(in, part.node_of_task);
    double mx = 0;
    for (double b : busy) mx = std::max(mx, b);
    CHECK(std::fabs(mx - part.period) <= 1e-12 * std::max(1.0, mx), "partition: period matches node cost");
    auto r = dls::run_policy(in, dls::Policy::EFT);
    CHECK(r.partitioned && r.steady_period < r.cold_period, "EFT takes the steady partition");
  }
  // a p2p pair whose sizes disagree: both ends fail with the real error, not a timeout
  {
    dls::P2PMatcher<CpuOp> m(2);
    std::vector<float> a(4), b(5);
    CpuOp sop, rop;
    sop.buf = &a;
    rop.buf = &b;
    auto copy = [](CpuOp& s, CpuOp& r) {
      if (s.buf->size() != r.buf->size()) throw std::runtime_error("size mismatch");
    };
    const int64_t sid = m.post(true, 0, 1, sop, copy);
    bool threw = false;
    try {
      m.post(false, 1, 0, rop, copy);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw, "mismatched post throws");
    bool peer_threw = false;
    try {
      m.wait(sid, 5.0);
    } catch (const std::runtime_error& e) {
      peer_threw = std::string(e.what()).find("size mismatch") != std::string::npos;
    }
    CHECK(peer_threw, "the counterpart's wait reports the size mismatch");
    CHECK(m.outstanding() == 0, "p2p: %lld ops left after a failed match (the posting op leaked)",
          (long long)m.outstanding());
  }
  // the step runner's action loop over the loopback pairing: 2 / 4 / 8 rank threads
  for (int world : {2, 4, 8}) p2p_pipeline(world, 4, 257, 20);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t, instances, seed);
  for (auto& th : pool) th.join();
  const int f = g_failures.load();
  std::printf("core_selftest: %d threads x %d instances x 5 policies: %s (%d failures)\n", threads, instances,
              f ? "FAILED" : "ok", f);
  return f ? 1 : 0;
}
