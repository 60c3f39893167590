// Native scheduling core — see scheduler.h for the behavioural contract.
#include "scheduler.h"

#include "partition.h"

#include <algorithm>
#include <cmath>
#include <deque>
#include <limits>
#include <numeric>
#include <stdexcept>

namespace dls {

namespace {

// EFT memory-fit slack (GB): fractional 'bytes' parameter costs summed in different
// orders differ by a few ulps; 1e-9 GB = 1 byte.
constexpr double kEftTol = 1e-9;

// Kahn order over the known dependency edges. Tasks on a cycle are appended at the
// end (they can never become ready, the reference would recurse forever on them).
std::vector<int> topo_order(const Instance& I, std::vector<std::vector<int>>& dependents) {
  const int T = static_cast<int>(I.task_ids.size());
  dependents.assign(T, {});
  std::vector<int> indeg(T, 0);
  for (int t = 0; t < T; ++t) {
    for (int d : I.deps[t]) {
      if (d < 0) continue;
      dependents[d].push_back(t);  // multiplicity kept (reference appends per occurrence)
      ++indeg[t];
    }
  }
  std::vector<int> order;
  order.reserve(T);
  std::deque<int> q;
  for (int t = 0; t < T; ++t)
    if (indeg[t] == 0) q.push_back(t);
  while (!q.empty()) {
    int t = q.front();
    q.pop_front();
    order.push_back(t);
    for (int d : dependents[t])
      if (--indeg[d] == 0) q.push_back(d);
  }
  if (static_cast<int>(order.size()) != T) {
    std::vector<char> seen(T, 0);
    for (int t : order) seen[t] = 1;
    for (int t = 0; t < T; ++t)
      if (!seen[t]) order.push_back(t);
  }
  return order;
}

struct Sched {
  const Instance& I;
  const int T, P, N;
  Result R;

  std::vector<char> pending;
  int n_pending = 0;
  std::vector<int> remaining;   // distinct known deps not yet completed
  std::vector<char> unknown;    // has a dependency that is not a task
  std::vector<std::vector<int>> dependents_multi;  // with multiplicity (urgency)
  std::vector<std::vector<int>> dependents;        // distinct
  std::set<int> live_ready;     // pending tasks whose deps are all completed, right now
  std::vector<int> ready_need;  // per param: #tasks in live_ready that need it

  std::vector<double> avail;
  std::vector<std::vector<char>> cached;
  std::vector<std::vector<int>> cached_list;
  std::vector<std::vector<int>> cached_pos;
  std::vector<std::vector<int>> node_completed;
  std::vector<std::deque<int>> last_used;
  std::vector<char> node_used;
  int round = 0;

  // MRU state
  std::vector<int> usage;
  std::vector<int> last_step;
  int time_step = 0;
  std::vector<int> name_rank;  // lexicographic rank of each param name (tie-break)
  std::vector<int> forced;     // EFT: node per task fixed by the steady partition (empty: free)

  explicit Sched(const Instance& inst)
      : I(inst),
        T(static_cast<int>(inst.task_ids.size())),
        P(static_cast<int>(inst.param_names.size())),
        N(static_cast<int>(inst.node_ids.size())) {
    pending.assign(T, 1);
    n_pending = T;
    remaining.assign(T, 0);
    unknown.assign(T, 0);
    dependents_multi.assign(T, {});
    dependents.assign(T, {});
    ready_need.assign(P, 0);
    for (int t = 0; t < T; ++t) {
      std::vector<int> ds;
      for (int d : I.deps[t]) {
        if (d < 0) {
          unknown[t] = 1;
          continue;
        }
        dependents_multi[d].push_back(t);
        ds.push_back(d);
      }
      std::sort(ds.begin(), ds.end());
      ds.erase(std::unique(ds.begin(), ds.end()), ds.end());
      remaining[t] = static_cast<int>(ds.size());
      for (int d : ds) dependents[d].push_back(t);
    }
    for (int t = 0; t < T; ++t)
      if (remaining[t] == 0 && !unknown[t]) make_live_ready(t);
    avail = I.node_mem;
    cached.assign(N, std::vector<char>(P, 0));
    cached_list.assign(N, {});
    cached_pos.assign(N, std::vector<int>(P, -1));
    node_completed.assign(N, {});
    last_used.assign(N, {});
    node_used.assign(N, 0);
    usage.assign(P, 0);
    last_step.assign(P, -1);
    std::vector<int> idx(P);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(),
              [&](int a, int b) { return I.param_names[a] < I.param_names[b]; });
    name_rank.assign(P, 0);
    for (int r = 0; r < P; ++r) name_rank[idx[r]] = r;
    R.assigned_node.assign(T, -1);
    R.completed.assign(T, 0);
    R.failed.assign(T, 0);
    R.schedule.assign(N, {});
  }

  void make_live_ready(int t) {
    live_ready.insert(t);
    for (int p : I.params[t]) ++ready_need[p];
  }
  void leave_pending(int t) {
    if (!pending[t]) return;
    pending[t] = 0;
    --n_pending;
    auto it = live_ready.find(t);
    if (it != live_ready.end()) {
      live_ready.erase(it);
      for (int p : I.params[t]) --ready_need[p];
    }
  }

  // --- memory model (schedulers.py:63-76) ---
  double load_cost(int t, int n) const {
    double s = 0.0;
    for (int p : I.params[t])
      if (!cached[n][p]) s += I.param_cost[p];
    return s;
  }
  int n_missing(int t, int n) const {
    int k = 0;
    for (int p : I.params[t])
      if (!cached[n][p]) ++k;
    return k;
  }
  int n_hit(int t, int n) const { return static_cast<int>(I.params[t].size()) - n_missing(t, n); }
  double requirement(int t, int n) const { return I.mem[t] + load_cost(t, n); }
  bool fits(int t, int n) const { return requirement(t, n) <= avail[n]; }

  void cache_add(int n, int p) {
    cached[n][p] = 1;
    cached_pos[n][p] = static_cast<int>(cached_list[n].size());
    cached_list[n].push_back(p);
  }
  void cache_remove(int n, int p) {
    cached[n][p] = 0;
    int pos = cached_pos[n][p];
    int last = cached_list[n].back();
    cached_list[n][pos] = last;
    cached_pos[n][last] = pos;
    cached_list[n].pop_back();
    cached_pos[n][p] = -1;
  }

  // --- assign = execute (schedulers.py:78-126) ---
  // ``tol``: slack for the accumulated rounding of fractional parameter costs. The
  // reference policies compare exactly (schedulers.py:66-76, tol = 0); EFT's dry-run
  // eviction sums the same costs in another order, so it passes a small tolerance.
  bool assign(int t, int n, double tol = 0.0) {
    if (requirement(t, n) > avail[n] + tol) return false;
    for (int p : I.params[t]) {
      if (cached[n][p]) continue;
      cache_add(n, p);
      avail[n] -= I.param_cost[p];
      R.events.push_back({round, static_cast<int>(Action::LOAD), n, p});
    }
    R.assigned_node[t] = n;
    avail[n] -= I.mem[t];
    leave_pending(t);
    for (int p : I.params[t]) {
      last_used[n].push_back(p);
      if (last_used[n].size() > 10) last_used[n].pop_front();
    }
    R.events.push_back({round, static_cast<int>(Action::RUN), n, t});
    if (!node_used[n]) {
      node_used[n] = 1;
      R.node_first_use_order.push_back(n);
    }
    R.schedule[n].push_back(t);
    complete(t, n);
    return true;
  }

  void complete(int t, int n) {
    R.completed[t] = 1;
    node_completed[n].push_back(t);
    avail[n] += I.mem[t];
    for (int d : dependents[t]) {
      if (--remaining[d] == 0 && pending[d] && !unknown[d]) make_live_ready(d);
    }
  }

  void fail(int t) {
    R.failed[t] = 1;
    leave_pending(t);
    R.events.push_back({round, static_cast<int>(Action::FAIL), -1, t});
  }

  void fail_all_pending() {
    for (int t = 0; t < T; ++t)
      if (pending[t]) fail(t);
  }

  std::vector<int> ready_snapshot() const { return std::vector<int>(live_ready.begin(), live_ready.end()); }

  // --- MRU eviction (schedulers.py:383-442) ---
  double eviction_score(int p) const {
    double s = 0.0;
    s += static_cast<double>(usage[p] * 10);
    if (last_step[p] >= 0) s += 100.0 / static_cast<double>(time_step - last_step[p] + 1);
    for (int k = 0; k < ready_need[p]; ++k) s += 1000;
    return s;
  }

  bool evict_for(int n, int t) {
    const double shortage = requirement(t, n) - avail[n];
    if (shortage <= 0) return true;
    std::vector<char> needed(P, 0);
    for (int p : I.params[t]) needed[p] = 1;
    std::vector<std::pair<double, int>> cand;
    for (int p : cached_list[n])
      if (!needed[p]) cand.emplace_back(eviction_score(p), p);
    std::sort(cand.begin(), cand.end(), [&](const auto& a, const auto& b) {
      if (a.first != b.first) return a.first < b.first;
      return name_rank[a.second] < name_rank[b.second];
    });
    double freed = 0;
    std::vector<int> evicted;
    for (const auto& c : cand) {
      if (freed >= shortage) break;
      cache_remove(n, c.second);
      avail[n] += I.param_cost[c.second];
      freed += I.param_cost[c.second];
      evicted.push_back(c.second);
    }
    if (freed >= shortage) {
      for (int p : evicted) R.events.push_back({round, static_cast<int>(Action::EVICT), n, p});
      return true;
    }
    for (int p : evicted) {
      cache_add(n, p);
      avail[n] -= I.param_cost[p];
    }
    return false;
  }

  // --- reference policies ---
  void run_reference(Policy pol) {
    std::vector<int> depth;
    std::vector<double> blevel;
    if (pol == Policy::DFS) depth = depth_from_sources(I);
    if (pol == Policy::CRITICAL) blevel = bottom_level(I);
    const int max_iter = T * 2;
    int iterations = 0;
    while (n_pending > 0 && iterations < max_iter) {
      ++iterations;
      round = iterations;
      if (pol == Policy::MRU) ++time_step;
      std::vector<int> ready = ready_snapshot();
      if (ready.empty()) break;
      if (pol == Policy::DFS) {
        std::stable_sort(ready.begin(), ready.end(), [&](int a, int b) { return depth[a] > depth[b]; });
      } else if (pol == Policy::CRITICAL) {
        std::stable_sort(ready.begin(), ready.end(), [&](int a, int b) { return blevel[a] > blevel[b]; });
      } else if (pol == Policy::MRU) {
        std::vector<int> urg(T, 0);
        for (int t : ready) {
          int u = 0;
          for (int d : dependents_multi[t])
            if (pending[d]) ++u;
          urg[t] = u;
        }
        std::stable_sort(ready.begin(), ready.end(), [&](int a, int b) { return urg[a] > urg[b]; });
      }
      bool progressed = false;
      for (int t : ready) {
        if (!pending[t]) continue;
        int best = -1;
        if (pol == Policy::DFS) {
          double maxm = -1;
          for (int n = 0; n < N; ++n)
            if (fits(t, n) && avail[n] > maxm) {
              best = n;
              maxm = avail[n];
            }
        } else if (pol == Policy::GREEDY) {
          double min_load = std::numeric_limits<double>::infinity();
          double best_av = 0;
          for (int n = 0; n < N; ++n) {
            if (!fits(t, n)) continue;
            const double k = n_missing(t, n);
            if (k < min_load || (k == min_load && avail[n] > best_av)) {
              best = n;
              min_load = k;
              best_av = avail[n];
            }
          }
        } else if (pol == Policy::CRITICAL) {
          double best_speed = 0;
          for (int n = 0; n < N; ++n)
            if (fits(t, n) && I.node_speed[n] > best_speed) {
              best = n;
              best_speed = I.node_speed[n];
            }
        } else {  // MRU
          double best_score = -std::numeric_limits<double>::infinity();
          for (int n = 0; n < N; ++n) {
            double score = 0.0;
            score += static_cast<double>(n_hit(t, n) * 20);
            if (fits(t, n)) {
              score += avail[n];
            } else if (evict_for(n, t)) {  // NB: probe evicts for real
              score += 5;
            } else {
              continue;
            }
            score -= static_cast<double>(node_completed[n].size()) * 0.5;
            if (score > best_score) {
              best_score = score;
              best = n;
            }
          }
          if (best >= 0 && !fits(t, best)) evict_for(best, t);
        }
        if (best >= 0) {
          if (assign(t, best)) {
            progressed = true;
            if (pol == Policy::MRU) {
              for (int p : I.params[t]) {
                ++usage[p];
                last_step[p] = time_step;
              }
            }
          }
        } else {
          fail(t);
        }
      }
      if (!progressed) {
        fail_all_pending();
        break;
      }
    }
    R.rounds = iterations;
  }

  // --- EFT: transfer-aware earliest-finish-time list scheduling (new policy) ---
  // Event-driven (no rounds): the highest upward-rank ready task is placed on the node
  // that finishes it earliest, accounting for (a) the node's serial compute timeline,
  // (b) cross-node input edges (link_lat + bytes/link_bw, one xGMI link per pair),
  // (c) parameter cache fills on the node's copy engine (prefetchable, overlapped with
  // compute) and (d) the per-node memory cap with least-useful-first eviction.
  void run_eft() {
    std::vector<double> out(T, 0.0);
    for (int t = 0; t < T; ++t) out[t] = I.out_size.empty() ? 0.0 : I.out_size[t];
    double mean_speed = 0;
    for (double s : I.node_speed) mean_speed += s;
    mean_speed = N > 0 ? mean_speed / N : 1.0;
    const double cross_frac = N > 1 ? double(N - 1) / N : 0.0;
    std::vector<std::vector<int>> deps_of_dummy;
    std::vector<int> order = topo_order(I, deps_of_dummy);
    std::vector<double> rank(T, 0.0);
    for (int i = T - 1; i >= 0; --i) {
      int t = order[i];
      double m = 0.0;
      for (int d : dependents[t]) {
        double c = cross_frac * (I.link_lat + out[t] / I.link_bw);
        m = std::max(m, c + rank[d]);
      }
      rank[t] = I.compute[t] / mean_speed + m;
    }
    std::vector<double> node_free(N, 0.0), copy_free(N, 0.0);
    std::vector<double> last_touch(P * static_cast<size_t>(std::max(N, 1)), -1.0);
    // next-use model for the eviction order (plan_eviction)
    eft_rank = rank;
    eft_users.assign(P, {});
    eft_first.assign(P, -std::numeric_limits<double>::infinity());
    eft_rmax = 0.0;
    for (int t = 0; t < T; ++t) {
      eft_rmax = std::max(eft_rmax, rank[t]);
      for (int p : I.params[t]) {
        eft_users[p].push_back(t);
        eft_first[p] = std::max(eft_first[p], rank[t]);
      }
    }
    R.start_time.assign(T, 0.0);
    R.finish_time.assign(T, 0.0);
    auto cmp = [&](int a, int b) {
      if (rank[a] != rank[b]) return rank[a] > rank[b];
      return a < b;
    };
    std::set<int, decltype(cmp)> ready(cmp);
    for (int t : live_ready) ready.insert(t);
    int step = 0;
    while (!ready.empty()) {
      int t = *ready.begin();
      ready.erase(ready.begin());
      round = ++step;
      ++time_step;
      int best = -1;
      double best_fin = std::numeric_limits<double>::infinity(), best_start = 0, best_fill = 0;
      std::vector<int> best_victims;
      for (int n = 0; n < N; ++n) {
        if (!forced.empty() && forced[t] >= 0 && forced[t] != n) continue;
        std::vector<int> victims;
        double need = requirement(t, n);
        if (need > avail[n] + kEftTol) {
          if (!plan_eviction(t, n, need - avail[n], last_touch, victims)) continue;
        }
        double data_ready = 0.0;
        for (int d : I.deps[t]) {
          if (d < 0) continue;
          double arr = R.finish_time[d];
          if (R.assigned_node[d] != n) arr += I.link_lat + out[d] / I.link_bw;
          data_ready = std::max(data_ready, arr);
        }
        const double fill = load_cost(t, n) / I.load_bw;
        const double fill_end = copy_free[n] + fill;
        const double start = std::max({node_free[n], data_ready, fill_end});
        const double fin = start + I.compute[t] / I.node_speed[n];
        if (fin < best_fin - 1e-15 || (std::fabs(fin - best_fin) <= 1e-15 && start < best_start)) {
          best = n;
          best_fin = fin;
          best_start = start;
          best_fill = fill_end;
          best_victims = victims;
        }
      }
      if (best < 0) {
        fail(t);
        continue;
      }
      for (int p : best_victims) {
        cache_remove(best, p);
        avail[best] += I.param_cost[p];
        R.events.push_back({round, static_cast<int>(Action::EVICT), best, p});
      }
      copy_free[best] = best_fill;
      node_free[best] = best_fin;
      R.start_time[t] = best_start;
      R.finish_time[t] = best_fin;
      // assign() completes the task and promotes dependents into live_ready; a
      // dependent whose last missing input was t is newly ready now. plan_eviction freed
      // >= shortage up to kEftTol, so this cannot fail; if it ever did, the task is
      // failed explicitly instead of being left pending with its dependents orphaned.
      if (!assign(t, best, kEftTol)) {
        fail(t);
        continue;
      }
      for (int p : I.params[t]) {
        last_touch[static_cast<size_t>(best) * P + p] = best_fin;
        ++usage[p];
        last_step[p] = time_step;
      }
      for (int d : dependents[t])
        if (remaining[d] == 0 && pending[d] && !unknown[d]) ready.insert(d);
    }
    // Invariant: a task still pending here has a failed, orphaned or unknown input.
    for (int t = 0; t < T; ++t)
      if (pending[t] && remaining[t] == 0 && !unknown[t])
        throw std::logic_error("EFT left a ready task unscheduled: " + I.task_ids[t]);
    R.rounds = step;
  }

  // EFT next-use model: upward rank per task (tasks run in decreasing rank), the tasks
  // using each parameter and the highest rank among them (its first use in a repetition).
  std::vector<double> eft_rank;
  std::vector<std::vector<int>> eft_users;
  std::vector<double> eft_first;
  double eft_rmax = 0.0;

  // Rank distance from task t to parameter p's next use: a pending user later in this
  // repetition, else (cyclic) p's first use in the next repetition of the DAG.
  double next_use_distance(int t, int p) const {
    const double now = eft_rank[t];
    double best = -std::numeric_limits<double>::infinity();
    for (int u : eft_users[p])
      if (pending[u] && u != t) best = std::max(best, eft_rank[u]);
    if (best > -std::numeric_limits<double>::infinity()) return std::max(0.0, now - best);
    return now + (eft_rmax - eft_first[p]) + 1e-12;
  }

  // Dry-run eviction. Never evicts this task's own params. Order:
  // * cyclic (default): cheapest refill per unit of budget freed first (param_refill), then
  //   farthest next use (Belady's rule under a repeating DAG): for a layer chain served step
  //   after step this keeps the FIRST layers' weights resident across the step boundary, so
  //   only the overflow is re-filled per step — least-recently-used order evicts every group
  //   before its next use and re-fills all of them;
  // * otherwise least useful first = not needed by any ready task, then oldest last use.
  // Ties: parameter name.
  bool plan_eviction(int t, int n, double shortage, const std::vector<double>& last_touch,
                     std::vector<int>& victims) const {
    std::vector<char> needed(P, 0);
    for (int p : I.params[t]) needed[p] = 1;
    std::vector<int> cand;
    for (int p : cached_list[n])
      if (!needed[p]) cand.push_back(p);
    if (I.cyclic) {
      // refill bytes per unit of budget freed: 1 when the budget counts real bytes; under
      // the reference's flat cost a 6 KB norm frees as much budget as a 77 MB embedding,
      // so the cheap-to-refill groups are streamed and the expensive ones stay resident
      std::vector<double> dist(P, 0.0), ratio(P, 1.0);
      const bool weighted = I.param_refill.size() == static_cast<size_t>(P);
      for (int p : cand) {
        dist[p] = next_use_distance(t, p);
        if (weighted && I.param_cost[p] > 0) ratio[p] = I.param_refill[p] / I.param_cost[p];
      }
      std::sort(cand.begin(), cand.end(), [&](int a, int b) {
        if (std::fabs(ratio[a] - ratio[b]) > 1e-6 * std::max(ratio[a], ratio[b])) return ratio[a] < ratio[b];
        if (dist[a] != dist[b]) return dist[a] > dist[b];
        return name_rank[a] < name_rank[b];
      });
    } else {
      std::sort(cand.begin(), cand.end(), [&](int a, int b) {
        const bool ra = ready_need[a] > 0, rb = ready_need[b] > 0;
        if (ra != rb) return rb;  // not-needed-now first
        const double la = last_touch[static_cast<size_t>(n) * P + a];
        const double lb = last_touch[static_cast<size_t>(n) * P + b];
        if (la != lb) return la < lb;
        return name_rank[a] < name_rank[b];
      });
    }
    double freed = 0;
    for (int p : cand) {
      if (freed >= shortage - kEftTol) break;
      victims.push_back(p);
      freed += I.param_cost[p];
    }
    return freed >= shortage - kEftTol;
  }

  Result finish() {
    R.nodes.resize(N);
    for (int n = 0; n < N; ++n) {
      R.nodes[n].available_memory = avail[n];
      R.nodes[n].cached = cached_list[n];
      std::sort(R.nodes[n].cached.begin(), R.nodes[n].cached.end());
      R.nodes[n].completed = node_completed[n];
      R.nodes[n].last_used.assign(last_used[n].begin(), last_used[n].end());
    }
    R.param_usage_count = usage;
    R.param_last_used = last_step;
    R.time_step = time_step;
    return std::move(R);
  }
};

void validate(const Instance& I) {
  const size_t T = I.task_ids.size();
  if (I.mem.size() != T || I.compute.size() != T || I.deps.size() != T || I.params.size() != T)
    throw std::invalid_argument("task arrays have inconsistent lengths");
  if (I.param_cost.size() != I.param_names.size())
    throw std::invalid_argument("param_cost/param_names length mismatch");
  if (I.node_mem.size() != I.node_ids.size() || I.node_speed.size() != I.node_ids.size())
    throw std::invalid_argument("node arrays have inconsistent lengths");
  if (!I.out_size.empty() && I.out_size.size() != T) throw std::invalid_argument("out_size length mismatch");
  if (!I.real_time.empty() && I.real_time.size() != T) throw std::invalid_argument("real_time length mismatch");
  const int P = static_cast<int>(I.param_names.size());
  for (size_t t = 0; t < T; ++t) {
    for (int d : I.deps[t])
      if (d >= static_cast<int>(T)) throw std::invalid_argument("dependency index out of range");
    for (int p : I.params[t])
      if (p < 0 || p >= P) throw std::invalid_argument("param index out of range");
  }
}

}  // namespace

std::vector<int> depth_from_sources(const Instance& I) {
  std::vector<std::vector<int>> dependents;
  std::vector<int> order = topo_order(I, dependents);
  const int T = static_cast<int>(I.task_ids.size());
  std::vector<int> depth(T, 0);
  for (int t : order) {
    if (I.deps[t].empty()) {
      depth[t] = 0;
      continue;
    }
    int m = 0;
    bool any = false;
    for (int d : I.deps[t]) {
      if (d < 0) continue;
      m = any ? std::max(m, depth[d]) : depth[d];
      any = true;
    }
    depth[t] = 1 + (any ? m : 0);
  }
  return depth;
}

std::vector<double> bottom_level(const Instance& I) {
  std::vector<std::vector<int>> dependents;
  std::vector<int> order = topo_order(I, dependents);
  const int T = static_cast<int>(I.task_ids.size());
  std::vector<double> bl(T, 0.0);
  for (int i = T - 1; i >= 0; --i) {
    const int t = order[i];
    if (dependents[t].empty()) {
      bl[t] = I.compute[t];
      continue;
    }
    double m = -std::numeric_limits<double>::infinity();
    for (int d : dependents[t]) m = std::max(m, bl[d]);
    bl[t] = I.compute[t] + m;
  }
  return bl;
}

// EFT: the cold earliest-finish-time pass, or — when the DAG repeats (cyclic), runs on
// several GPUs and the cold pass leaves parameter groups to re-fill every step — the
// steady-state partition (partition.h) if its modelled step period is >= 2 % shorter. The
// partition only fixes each task's GPU; the list scheduler then re-runs with that
// constraint, so loads, evictions and the timeline come from the same memory accounting.
static Result run_eft_steady(const Instance& inst) {
  Sched cold_s(inst);
  cold_s.run_eft();
  Result cold = cold_s.finish();
  const int N = static_cast<int>(inst.node_ids.size());
  if (!inst.cyclic || !inst.steady || N < 1) return cold;
  std::vector<double> refill;
  std::vector<double> busy = steady_node_cost(inst, cold.assigned_node, &refill);
  cold.cold_period = cold.steady_period = *std::max_element(busy.begin(), busy.end());
  if (N < 2 || std::accumulate(refill.begin(), refill.end(), 0.0) <= 0.0) return cold;
  Partition part = steady_partition(inst);
  if (!part.feasible || !(part.period < cold.cold_period * (1.0 - 0.02))) return cold;
  Sched s(inst);
  s.forced = part.node_of_task;
  s.run_eft();
  Result r = s.finish();
  const auto done = [](const Result& x) { return std::accumulate(x.completed.begin(), x.completed.end(), 0); };
  if (done(r) < done(cold)) return cold;
  busy = steady_node_cost(inst, r.assigned_node, nullptr);
  r.cold_period = cold.cold_period;
  r.steady_period = *std::max_element(busy.begin(), busy.end());
  r.partitioned = true;
  r.stage_node = part.stage_node;
  r.stage_busy = part.stage_busy;
  r.stage_refill_gb = part.stage_refill_gb;
  return r;
}

Result run_policy(const Instance& inst, Policy policy) {
  validate(inst);
  if (policy == Policy::EFT) return run_eft_steady(inst);
  Sched s(inst);
  s.run_reference(policy);
  return s.finish();
}

void replay_with_deps(const Instance& I, const std::vector<std::vector<int>>& schedule,
                      std::vector<double>& start, std::vector<double>& finish, bool with_transfers) {
  const int T = static_cast<int>(I.task_ids.size());
  const int N = static_cast<int>(schedule.size());
  start.assign(T, std::nan(""));
  finish.assign(T, std::nan(""));
  std::vector<int> loc(T, -1);
  for (int n = 0; n < N; ++n)
    for (int t : schedule[n]) loc[t] = n;
  std::vector<size_t> head(N, 0);
  std::vector<double> node_free(N, 0.0);
  bool progress = true;
  while (progress) {
    progress = false;
    for (int n = 0; n < N; ++n) {
      while (head[n] < schedule[n].size()) {
        const int t = schedule[n][head[n]];
        double ready = 0.0;
        bool ok = true;
        for (int d : I.deps[t]) {
          if (d < 0 || std::isnan(finish[d])) {
            ok = false;
            break;
          }
          double arr = finish[d];
          if (with_transfers && loc[d] != n) {
            const double bytes = I.out_size.empty() ? 0.0 : I.out_size[d];
            arr += I.link_lat + bytes / I.link_bw;
          }
          ready = std::max(ready, arr);
        }
        if (!ok) break;
        const double speed = I.node_speed.empty() ? 1.0 : I.node_speed[n];
        start[t] = std::max(node_free[n], ready);
        finish[t] = start[t] + I.compute[t] / speed;
        node_free[n] = finish[t];
        ++head[n];
        progress = true;
      }
    }
  }
}

}  // namespace dls
