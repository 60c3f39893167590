// Steady-state min-max pipeline partition — see partition.h for the model.
#include "partition.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <functional>
#include <limits>
#include <numeric>
#include <queue>

namespace dls {

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();
constexpr double kTol = 1e-9;

struct Model {
  const Instance& I;
  int T, P, N;
  std::vector<double> rt;        // real seconds per task on a speed-1 node
  std::vector<double> refill;    // GB a refill of each parameter moves
  std::vector<int> prio;         // parameter ids, keep-first order
  std::vector<int> prio_rank;    // parameter id -> position in prio
  std::vector<double> foot;      // per task: budget units of its own parameters
  std::vector<double> edge;      // per task: cost of sending its output once (s)

  explicit Model(const Instance& inst)
      : I(inst),
        T(static_cast<int>(inst.task_ids.size())),
        P(static_cast<int>(inst.param_names.size())),
        N(static_cast<int>(inst.node_ids.size())) {
    rt = I.real_time.size() == static_cast<size_t>(T) ? I.real_time : I.compute;
    refill = I.param_refill.size() == static_cast<size_t>(P) ? I.param_refill : I.param_cost;
    std::vector<double> ratio(P, 1.0);
    for (int p = 0; p < P; ++p)
      if (I.param_cost[p] > 0) ratio[p] = refill[p] / I.param_cost[p];
    prio.resize(P);
    std::iota(prio.begin(), prio.end(), 0);
    std::stable_sort(prio.begin(), prio.end(), [&](int a, int b) {
      if (std::fabs(ratio[a] - ratio[b]) > 1e-6 * std::max(ratio[a], ratio[b])) return ratio[a] > ratio[b];
      if (refill[a] != refill[b]) return refill[a] > refill[b];
      return a < b;
    });
    prio_rank.assign(P, 0);
    for (int r = 0; r < P; ++r) prio_rank[prio[r]] = r;
    foot.assign(T, 0.0);
    edge.assign(T, 0.0);
    for (int t = 0; t < T; ++t) {
      for (int p : I.params[t]) foot[t] += I.param_cost[p];
      const double bytes = I.out_size.empty() ? 0.0 : I.out_size[t];
      edge[t] = I.link_lat + bytes / I.link_bw + I.p2p_host;
    }
  }

  double speed(int n) const { return I.node_speed.empty() || I.node_speed[n] <= 0 ? 1.0 : I.node_speed[n]; }

  // Streamed (re-filled) GB per step of a stage holding the parameter set `bits` (priority
  // ranks), or +inf if the stage cannot run under `cap` at all.
  double refill_gb(const std::vector<uint64_t>& bits, double sum_cost, double sum_refill, double mem_max,
                   double foot_max, double cap) const {
    const double room = cap - mem_max;
    if (sum_cost <= room + kTol) return 0.0;  // everything resident
    const double avail = room - foot_max;      // the streaming buffer takes a task's groups
    if (avail < -kTol) return kInf;
    double kept = 0.0, streamed = sum_refill;
    for (size_t w = 0; w < bits.size(); ++w) {
      uint64_t b = bits[w];
      while (b) {
        const int r = static_cast<int>(w * 64 + __builtin_ctzll(b));
        b &= b - 1;
        const int p = prio[r];
        if (kept + I.param_cost[p] <= avail + kTol) {
          kept += I.param_cost[p];
          streamed -= refill[p];
        }
      }
    }
    return std::max(streamed, 0.0);
  }
};

}  // namespace

std::vector<int> steady_order(const Instance& I) {
  const int T = static_cast<int>(I.task_ids.size());
  std::vector<std::vector<int>> dependents(T);
  std::vector<int> indeg(T, 0);
  for (int t = 0; t < T; ++t) {
    std::vector<int> ds;
    for (int d : I.deps[t])
      if (d >= 0) ds.push_back(d);
    std::sort(ds.begin(), ds.end());
    ds.erase(std::unique(ds.begin(), ds.end()), ds.end());
    for (int d : ds) dependents[d].push_back(t);
    indeg[t] = static_cast<int>(ds.size());
  }
  const std::vector<double>& rt = I.real_time.size() == static_cast<size_t>(T) ? I.real_time : I.compute;
  // upward rank (longest compute path to a sink), over a plain Kahn order
  std::vector<int> kahn;
  {
    std::vector<int> deg = indeg;
    std::vector<int> q;
    for (int t = 0; t < T; ++t)
      if (deg[t] == 0) q.push_back(t);
    for (size_t h = 0; h < q.size(); ++h)
      for (int d : dependents[q[h]])
        if (--deg[d] == 0) q.push_back(d);
    kahn = q;
  }
  std::vector<double> rank(T, 0.0);
  for (int i = static_cast<int>(kahn.size()) - 1; i >= 0; --i) {
    const int t = kahn[i];
    double m = 0.0;
    for (int d : dependents[t]) m = std::max(m, rank[d]);
    rank[t] = rt[t] + m;
  }
  auto later = [&](int a, int b) {  // priority queue: highest rank first, then lower index
    if (rank[a] != rank[b]) return rank[a] < rank[b];
    return a > b;
  };
  std::priority_queue<int, std::vector<int>, decltype(later)> ready(later);
  for (int t = 0; t < T; ++t)
    if (indeg[t] == 0) ready.push(t);
  std::vector<int> order;
  order.reserve(T);
  while (!ready.empty()) {
    const int t = ready.top();
    ready.pop();
    order.push_back(t);
    for (int d : dependents[t])
      if (--indeg[d] == 0) ready.push(d);
  }
  return order;  // tasks on a dependency cycle (never runnable) are left out
}

std::vector<double> steady_node_cost(const Instance& I, const std::vector<int>& node_of_task,
                                     std::vector<double>* refill_out) {
  Model M(I);
  std::vector<double> busy(M.N, 0.0), refill(M.N, 0.0);
  for (int n = 0; n < M.N; ++n) {
    std::vector<uint64_t> bits((M.P + 63) / 64, 0);
    std::vector<char> in(M.P, 0);
    double sc = 0, sr = 0, mem = 0, foot = 0, comp = 0, comm = 0;
    bool any = false;
    std::vector<char> sent_to(static_cast<size_t>(M.T) * M.N, 0);
    std::vector<char> got(M.T, 0);
    for (int t = 0; t < M.T; ++t) {
      if (node_of_task[t] != n) continue;
      any = true;
      comp += M.rt[t] / M.speed(n);
      mem = std::max(mem, I.mem[t]);
      foot = std::max(foot, M.foot[t]);
      for (int p : I.params[t]) {
        if (in[p]) continue;
        in[p] = 1;
        sc += I.param_cost[p];
        sr += M.refill[p];
        const int r = M.prio_rank[p];
        bits[r / 64] |= uint64_t(1) << (r % 64);
      }
      for (int d : I.deps[t]) {  // received inputs: one transfer per distinct producer
        if (d < 0 || node_of_task[d] < 0 || node_of_task[d] == n || got[d]) continue;
        got[d] = 1;
        comm += M.edge[d];
      }
    }
    // sent outputs: one transfer per (producer on n, consumer node)
    for (int t = 0; t < M.T; ++t) {
      const int c = node_of_task[t];
      if (c < 0 || c == n) continue;
      for (int d : I.deps[t]) {
        if (d < 0 || node_of_task[d] != n) continue;
        char& s = sent_to[static_cast<size_t>(d) * M.N + c];
        if (!s) {
          s = 1;
          comm += M.edge[d];
        }
      }
    }
    if (!any) continue;
    refill[n] = M.refill_gb(bits, sc, sr, mem, foot, I.node_mem[n]);
    busy[n] = comp + refill[n] / I.load_bw + comm;
  }
  if (refill_out) *refill_out = refill;
  return busy;
}

Partition steady_partition(const Instance& I, int max_stages, int min_stages) {
  Model M(I);
  Partition out;
  out.order = steady_order(I);
  const int T = static_cast<int>(out.order.size());
  const int N = M.N;
  if (T == 0 || N == 0) return out;
  const int K = max_stages > 0 ? std::min(max_stages, N) : N;
  std::vector<int> pos(M.T, -1);
  for (int i = 0; i < T; ++i) pos[out.order[i]] = i;
  // last position at which each task's output is consumed
  std::vector<int> last_use(M.T, -1);
  for (int i = 0; i < T; ++i)
    for (int d : I.deps[out.order[i]])
      if (d >= 0 && pos[d] >= 0) last_use[d] = std::max(last_use[d], i);

  // Clean cut points: positions crossed by the fewest distinct producers (in a transformer
  // DAG the residual stream alone, at every attention / MLP half-layer boundary). A cut
  // anywhere else also splits a fused kernel pair (a norm folded into its GEMM, a residual
  // epilogue), which the per-task costs do not see. Cuts are restricted to them when the
  // partition stays feasible that way.
  std::vector<int> crossing(T + 2, 0);
  for (int i = 0; i < T; ++i) {
    const int u = out.order[i];
    if (last_use[u] > i) {
      ++crossing[i + 1];
      --crossing[last_use[u] + 1];
    }
  }
  for (int i = 1; i <= T; ++i) crossing[i] += crossing[i - 1];
  int min_cross = std::numeric_limits<int>::max();
  for (int i = 1; i < T; ++i) min_cross = std::min(min_cross, crossing[i]);
  // cuts that would split a fused kernel chain (Instance::fuse_into) are never taken
  std::vector<int> splits(T + 2, 0);
  if (I.fuse_into.size() == static_cast<size_t>(M.T))
    for (int t = 0; t < M.T; ++t) {
      const int c = I.fuse_into[t];
      if (c < 0 || pos[t] < 0 || pos[c] < 0) continue;
      const int lo = std::min(pos[t], pos[c]), hi = std::max(pos[t], pos[c]);
      ++splits[lo + 1];
      --splits[hi + 1];
    }
  for (int i = 1; i <= T; ++i) splits[i] += splits[i - 1];
  std::vector<char> allowed(T + 1, 1), clean(T + 1, 0);
  clean[0] = 1;
  for (int i = 1; i < T; ++i) {
    allowed[i] = splits[i] == 0;
    clean[i] = allowed[i] && crossing[i] <= min_cross;
  }

  // cost[n][i*(T+1)+j]: busy time of stage [i, j) on node n (distinct nodes only)
  std::vector<int> rep(N);  // node -> representative node with the same cap and speed
  for (int n = 0; n < N; ++n) {
    rep[n] = n;
    for (int m = 0; m < n; ++m)
      if (I.node_mem[m] == I.node_mem[n] && M.speed(m) == M.speed(n)) {
        rep[n] = rep[m];
        break;
      }
  }
  const size_t W = static_cast<size_t>(T + 1);
  // The stage tables hold (T+1)^2 doubles each: two per distinct node plus comp / comm. Beyond
  // kMaxTableBytes (multi-replica or heterogeneous DAGs of thousands of tasks) the partition is
  // not attempted and EFT keeps its cold plan — GBs of tables and O(T^2 N) time per plan would
  // cost more than the steady-state refills they could save.
  {
    constexpr double kMaxTableBytes = 512.0 * (1 << 20);
    int distinct = 0;
    for (int n = 0; n < N; ++n) distinct += rep[n] == n;
    if (double(2 * distinct + 2) * double(W) * double(W) * sizeof(double) > kMaxTableBytes) return out;
  }
  std::vector<std::vector<double>> cost(N);
  std::vector<std::vector<double>> refill_tab(N);
  for (int n = 0; n < N; ++n)
    if (rep[n] == n) {
      cost[n].assign(W * W, kInf);
      refill_tab[n].assign(W * W, 0.0);
    }
  std::vector<uint64_t> bits((M.P + 63) / 64);
  std::vector<char> in(M.P);
  std::vector<int> seen(M.T, -1);
  std::vector<double> rem(T + 2);
  std::vector<double> comp_tab(W * W, 0.0), comm_tab(W * W, 0.0);
  for (int i = 0; i < T; ++i) {
    std::fill(bits.begin(), bits.end(), 0);
    std::fill(in.begin(), in.end(), 0);
    std::fill(rem.begin(), rem.end(), 0.0);
    double sc = 0, sr = 0, mem = 0, foot = 0, comp = 0, comm_in = 0, comm_out = 0;
    for (int j = i + 1; j <= T; ++j) {
      const int t = out.order[j - 1];
      comp += M.rt[t];
      mem = std::max(mem, I.mem[t]);
      foot = std::max(foot, M.foot[t]);
      for (int p : I.params[t]) {
        if (in[p]) continue;
        in[p] = 1;
        sc += I.param_cost[p];
        sr += M.refill[p];
        const int r = M.prio_rank[p];
        bits[r / 64] |= uint64_t(1) << (r % 64);
      }
      for (int d : I.deps[t]) {
        if (d < 0 || pos[d] < 0 || pos[d] >= i || seen[d] == i) continue;
        seen[d] = i;  // received once per distinct producer before the stage
        comm_in += M.edge[d];
      }
      if (last_use[t] >= j) {  // consumed after the stage: sent once
        comm_out += M.edge[t];
        rem[last_use[t] + 1] += M.edge[t];
      }
      comm_out -= rem[j];
      rem[j] = 0.0;
      const double comm = comm_in + std::max(comm_out, 0.0);
      comp_tab[i * W + j] = comp;
      comm_tab[i * W + j] = comm;
      for (int n = 0; n < N; ++n) {
        if (rep[n] != n) continue;
        const double rg = M.refill_gb(bits, sc, sr, mem, foot, I.node_mem[n]);
        refill_tab[n][i * W + j] = rg;
        cost[n][i * W + j] = std::isinf(rg) ? kInf : comp / M.speed(n) + rg / I.load_bw + comm;
      }
    }
  }

  // candidate node orders for the pipeline stages
  std::vector<std::vector<int>> orders;
  auto add_order = [&](std::vector<int> o) {
    if (std::find(orders.begin(), orders.end(), o) == orders.end()) orders.push_back(std::move(o));
  };
  std::vector<int> ident(N);
  std::iota(ident.begin(), ident.end(), 0);
  add_order(ident);
  auto by = [&](std::function<bool(int, int)> less) {
    std::vector<int> o = ident;
    std::stable_sort(o.begin(), o.end(), less);
    add_order(o);
  };
  by([&](int a, int b) { return I.node_mem[a] > I.node_mem[b]; });
  by([&](int a, int b) { return I.node_mem[a] < I.node_mem[b]; });
  by([&](int a, int b) { return M.speed(a) > M.speed(b); });

  // Two passes: clean cuts only, then every cut that splits no fused chain; the second pass
  // (multi-producer cuts: more transfers, already in the edge costs) is taken only for a >= 3 %
  // shorter period, or when the clean cuts cannot make a feasible partition.
  double best = kInf;
  int best_k = 0;
  std::vector<int> best_cuts, best_nodes;
  double clean_best = kInf;
  // (without fusion chains (Instance::fuse_into) any non-clean cut may split a fused kernel
  // pair, so the finer pass only runs when the clean cuts are infeasible)
  const bool know_fusion = I.fuse_into.size() == static_cast<size_t>(M.T);
  for (int only_clean = 1; only_clean >= 0; --only_clean) {
  if (!only_clean && !know_fusion && best_k > 0) break;
  if (!only_clean) {
    clean_best = best;
    if (std::isfinite(best)) best *= 0.97;  // what the finer cuts must beat
  }
  const std::vector<char>& cut_ok = only_clean ? clean : allowed;
  for (const auto& o : orders) {
    // f[k][j]: min over cuts of the max stage busy covering positions [0, j) with k stages
    // (ties on the max: the smaller sum of squared stage times, i.e. the non-bottleneck
    // stages evened out too)
    std::vector<std::vector<double>> f(K + 1, std::vector<double>(T + 1, kInf));
    std::vector<std::vector<double>> g(K + 1, std::vector<double>(T + 1, kInf));
    std::vector<std::vector<int>> arg(K + 1, std::vector<int>(T + 1, -1));
    f[0][0] = g[0][0] = 0.0;
    for (int k = 1; k <= K; ++k) {
      const std::vector<double>& c = cost[rep[o[k - 1]]];
      for (int j = 1; j <= T; ++j) {
        double bv = kInf, bg = kInf;
        int bi = -1;
        for (int i = k - 1; i < j; ++i) {
          if (std::isinf(f[k - 1][i]) || !cut_ok[i]) continue;
          const double cij = c[i * W + j];
          const double v = std::max(f[k - 1][i], cij);
          const double sq = g[k - 1][i] + cij * cij;
          if (v < bv * (1.0 - 1e-9) || (v <= bv * (1.0 + 1e-9) && sq < bg)) {
            bv = v;
            bg = sq;
            bi = i;
          }
        }
        f[k][j] = bv;
        g[k][j] = bg;
        arg[k][j] = bi;
      }
    }
    for (int k = std::max(1, std::min(min_stages, K)); k <= K; ++k) {
      const double v = f[k][T];
      // another stage (GPU) has to buy a real improvement: 0.5 %
      const bool better = best_k == 0 ? std::isfinite(v) : (v < best * (1.0 - 5e-3) ||
                                                            (k == best_k && v < best - kTol));
      if (!better) continue;
      best = v;
      best_k = k;
      best_cuts.assign(k + 1, 0);
      best_cuts[k] = T;
      for (int kk = k, j = T; kk >= 1; --kk) {
        j = arg[kk][j];
        best_cuts[kk - 1] = j;
      }
      best_nodes.assign(o.begin(), o.begin() + k);
    }
  }
  }
  if (best_k == 0) return out;
  (void)clean_best;
  out.feasible = true;
  out.node_of_task.assign(M.T, -1);
  for (int s = 0; s < best_k; ++s) {
    const int a = best_cuts[s], b = best_cuts[s + 1], n = best_nodes[s];
    out.stage_node.push_back(n);
    out.stage_begin.push_back(a);
    for (int q = a; q < b; ++q) out.node_of_task[out.order[q]] = n;
    const size_t ij = static_cast<size_t>(a) * W + b;
    out.stage_busy.push_back(cost[rep[n]][ij]);
    out.stage_compute.push_back(comp_tab[ij] / M.speed(n));
    out.stage_refill_gb.push_back(refill_tab[rep[n]][ij]);
    out.stage_comm.push_back(comm_tab[ij]);
  }
  out.period = *std::max_element(out.stage_busy.begin(), out.stage_busy.end());
  out.stage_begin.push_back(T);
  return out;
}

}  // namespace dls
