// Native DAG scheduling core for distributed_llm_scheduler_amd.
//
// Behavioural contract mirrors the reference policies
// (/root/reference/schedulers.py:31-525) but the implementation is new:
//   * tasks/params/nodes are interned to dense integer ids,
//   * readiness is tracked incrementally (remaining-dependency counters and an
//     ordered live-ready set) instead of the reference's O(|pending|*deg) rescans
//     (schedulers.py:55-61),
//   * depth / bottom-level are computed by iterative topological DP instead of the
//     recursive memoised walks that overflow at ~900-deep chains
//     (schedulers.py:140-152, 301-321),
//   * MRU's "needed by a currently-ready pending task" term (schedulers.py:395-400)
//     is a per-parameter live counter, O(1) per lookup,
//   * every placement decision is emitted as an action trace (LOAD / EVICT / RUN /
//     FAIL) that the GPU executor replays as real HBM traffic.
//
// Tie-break order is task insertion order (deterministic). The reference iterates a
// Python set of strings (hash-seed dependent); the Python engine in
// core/schedulers.py (hash_order_compat=True) can replay that order when bit-exact hash-order replay is needed.
#pragma once

#include <cstdint>
#include <set>
#include <string>
#include <vector>

namespace dls {

enum class Policy : int { DFS = 0, GREEDY = 1, CRITICAL = 2, MRU = 3, EFT = 4 };

enum class Action : int { RUN = 0, LOAD = 1, EVICT = 2, FAIL = 3 };

struct Event {
  int round;
  int action;  // Action
  int node;    // -1 for FAIL
  int item;    // task index (RUN/FAIL) or param index (LOAD/EVICT)
};

struct Instance {
  std::vector<std::string> task_ids;
  std::vector<double> mem;      // activation/workspace (GB), freed on completion
  std::vector<double> compute;  // seconds on a speed-1.0 node
  std::vector<std::vector<int>> deps;    // -1 marks an id that is not a task
  std::vector<std::vector<int>> params;  // interned parameter ids
  std::vector<std::string> param_names;
  std::vector<double> param_cost;  // GB per parameter (0.5 everywhere in the reference model)
  std::vector<std::string> node_ids;
  std::vector<double> node_mem;
  std::vector<double> node_speed;
  // Only used by the EFT policy and the dependency-aware replay.
  std::vector<double> out_size;  // GB produced by each task (edge payload)
  double link_bw = 153.0;        // GB/s per xGMI link
  double link_lat = 5e-6;        // s per point-to-point message
  double load_bw = 50.0;         // GB/s for a parameter cache fill (H2D)
  // EFT eviction: true = the DAG repeats (one DAG per serving step; farthest next use,
  // counting the next repetition), false = least recently used among those no ready task needs
  bool cyclic = true;
  // Optional: bytes (GB) a refill of each parameter really moves, when the budget cost
  // model differs (the reference's flat 0.5 GB per parameter). Empty = param_cost.
  std::vector<double> param_refill;
  // Optional: real seconds per task on a speed-1.0 node (roofline of its FLOPs and bytes)
  // for the steady-state model, when `compute` is in other units (the reference's
  // constants). Empty = compute.
  std::vector<double> real_time;
  // EFT with cyclic = true: also plan the steady state (partition.h) and keep whichever of
  // the cold pass and the steady partition has the shorter modelled step period.
  bool steady = true;
  // Steady-state model only: host time per p2p transfer on each end (the step runner's
  // segment boundary at a receive, ~10-16 us measured; README "native step runner").
  double p2p_host = 10e-6;
  // Steady-state model only (optional): task -> the task whose fused kernel it runs in when
  // co-located (program lowering's fusion chains), -1 = none. A pipeline cut never splits one.
  std::vector<int> fuse_into;
};

struct NodeResult {
  double available_memory = 0.0;
  std::vector<int> cached;           // parameter ids resident at the end
  std::vector<int> completed;        // task ids in completion order
  std::vector<int> last_used;        // last <=10 params touched (reference deque maxlen=10)
};

struct Result {
  std::vector<int> assigned_node;  // -1 if not assigned
  std::vector<int> completed;
  std::vector<int> failed;
  std::vector<int> node_first_use_order;  // order in which nodes first received a task
  std::vector<std::vector<int>> schedule;  // per node, tasks in assignment order
  std::vector<NodeResult> nodes;
  std::vector<Event> events;
  int rounds = 0;
  // MRU statistics (schedulers.py:377-381)
  std::vector<int> param_usage_count;
  std::vector<int> param_last_used;  // -1 = never
  int time_step = 0;
  // EFT timeline (seconds) when Policy::EFT
  std::vector<double> start_time, finish_time;
  // EFT steady-state model (partition.h): modelled step period of the cold pass and of the
  // returned placement (s), whether the steady partition replaced the cold pass, and its
  // pipeline stages (node, busy s, re-filled GB per step).
  double cold_period = 0.0, steady_period = 0.0;
  bool partitioned = false;
  std::vector<int> stage_node;
  std::vector<double> stage_busy, stage_refill_gb;
};

Result run_policy(const Instance& inst, Policy policy);

// Dependency-respecting replay of a fixed placement: each node executes its list in
// order, a task starts when its node is free and every input has arrived
// (cross-node edges pay link_lat + out_size/link_bw). Returns per-task start/finish.
void replay_with_deps(const Instance& inst, const std::vector<std::vector<int>>& schedule,
                      std::vector<double>& start, std::vector<double>& finish, bool with_transfers);

// Iterative topological helpers (exposed for tests and the Python layer).
std::vector<int> depth_from_sources(const Instance& inst);
std::vector<double> bottom_level(const Instance& inst);

}  // namespace dls
