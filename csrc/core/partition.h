// Steady-state placement of ONE repeating DAG over N capped GPUs.
//
// The reference's experiment spreads one DAG over 2/4/8 memory-capped nodes
// (/root/reference/simulation.py:161-192, 375-376). Its policies decide each task once, as a
// cold single pass (schedulers.py:444-525); the executor, however, replays the placement
// every serving step. In that steady state a GPU's cost per step is its kernels plus the
// parameter groups it has to RE-FILL because its budget cannot keep them (host link, one
// per GPU, in parallel across GPUs) plus the p2p edges it sends and receives (one xGMI
// link per pair). Consecutive steps pipeline through the GPUs (a rank starts step k+1 as
// soon as its own part of step k and its sends are done), so the step period is the
// BUSIEST GPU's per-step time, not the sum along the chain.
//
// A cold earliest-finish-time pass never sees that: every parameter must be loaded once
// anyway, so an empty GPU never looks better and one GPU re-fills the overflow of the
// whole model every step while the others idle. steady_partition() instead minimises the
// modelled period over contiguous segments of a topological order (a pipeline of stages,
// one GPU each), by DP over the cut points (min-max partition), with:
//   stage busy  = sum(real_time)/speed + refill_gb/load_bw + edges in + edges out
//   refill_gb   = the bytes of the groups the stage's keep set cannot hold: groups kept
//                 greedily by refill bytes per budget unit (program.plan_keep_sets' rule),
//                 under budget = cap - largest activation - the largest per-task group
//                 footprint (the streaming buffer)
//   edges       = link_lat + bytes/link_bw per distinct producer crossing the cut.
#pragma once

#include <vector>

#include "scheduler.h"

namespace dls {

struct Partition {
  bool feasible = false;
  double period = 0.0;             // modelled steady-state step period (s)
  std::vector<int> order;          // the topological order the stages cut
  std::vector<int> node_of_task;   // node per task (-1: not placed)
  std::vector<int> stage_node;     // per stage, in pipeline order
  std::vector<int> stage_begin;    // first position in `order` (stage s = [begin[s], begin[s+1]))
  std::vector<double> stage_busy, stage_compute, stage_refill_gb, stage_comm;
};

// Per-node modelled cost of an arbitrary assignment (node per task; -1 = unplaced), with the
// same terms as a partition stage. Returns busy time per node; `refill_gb` per node.
std::vector<double> steady_node_cost(const Instance& I, const std::vector<int>& node_of_task,
                                     std::vector<double>* refill_gb = nullptr);

// Topological order used for the cut points: Kahn's algorithm releasing the highest
// upward rank first (ties: lower index), so replicas of one DAG interleave stage by stage.
std::vector<int> steady_order(const Instance& I);

// Best contiguous partition of steady_order(I) over at most `max_stages` of the N nodes
// (-1: N) and at least `min_stages` (pipeline placement asks for every GPU); another stage
// is only added for a >= 0.5 % shorter period.
Partition steady_partition(const Instance& I, int max_stages = -1, int min_stages = 1);

}  // namespace dls
