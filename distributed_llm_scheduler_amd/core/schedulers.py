"""Scheduling policies.

Public surface is reference-compatible (``/root/reference/schedulers.py``):
``BaseScheduler`` and the four policies ``DFSScheduler``, ``GreedyScheduler``,
``CriticalPathScheduler``, ``MRUScheduler`` with ``add_task`` / ``schedule()`` returning
``{node_id: [task_id, ...]}`` and the same mutable state (``completed_tasks``,
``failed_tasks``, ``pending_tasks``, ``param_locations``, per-node ``cached_params`` ...).

Two engines implement the policies:

* ``engine="native"`` (default) — the C++ core (csrc/core/scheduler.cpp): iterative
  depth / bottom-level (no RecursionError at ~900-deep chains), incremental
  readiness, O(1) MRU "needed-by-a-ready-task" lookups. Deterministic insertion-order
  tie-breaking.
* ``engine="python"`` — the same semantics in Python on top of the BaseScheduler
  primitives. With ``hash_order_compat=True`` the ready list is produced by iterating the
  ``pending_tasks`` set exactly like the reference (``schedulers.py:55-61``), so a run
  with the same ``PYTHONHASHSEED`` replays the reference bit-for-bit.

A fifth policy, :class:`EFTScheduler` ("XGMI-EFT"), is new: transfer- and memory-aware
earliest-finish-time list scheduling for the MI355X executor (native only).

Every run records an action trace in ``scheduler.events`` — ``(round, "LOAD"|"EVICT"|
"RUN"|"FAIL", node_id|None, item_id)`` — which the executor turns into real parameter
cache fills / evictions and kernel launches.
"""
from __future__ import annotations

import math
from collections import defaultdict, deque
from typing import Callable, Dict, List, Mapping, Optional, Sequence, Union

from .task import Node, Task
from . import native as _native

ACTIONS = ("RUN", "LOAD", "EVICT", "FAIL")
ParamCost = Union[float, Mapping[str, float], Callable[[str], float]]


def default_engine() -> str:
    return "native" if _native.available() else "python"


class BaseScheduler:
    """Registry, readiness, memory/parameter-cache accounting (reference C3-C8)."""

    #: native policy id; None for policies without a native implementation
    native_policy: Optional[int] = None
    name = "base"

    def __init__(self, nodes: Sequence[Node], *, engine: Optional[str] = None, param_cost: ParamCost = 0.5,
                 hash_order_compat: bool = False):
        self.nodes: Dict[str, Node] = {node.id: node for node in nodes}
        self.tasks: Dict[str, Task] = {}
        self.ready_queue: List[str] = []
        self.completed_tasks = set()
        self.failed_tasks = set()
        self.task_dependencies = defaultdict(list)  # dependents map (reverse edges), name kept for compat
        self.param_locations = defaultdict(set)
        self.pending_tasks = set()
        self._insertion: List[str] = []
        self.engine = engine or default_engine()
        self.param_cost = param_cost
        self.hash_order_compat = hash_order_compat
        self.events: List[tuple] = []
        self.rounds = 0
        self._round = 0

    # ---------------------------------------------------------------- registry
    def add_task(self, task: Task) -> None:
        if task.id not in self.tasks:
            self._insertion.append(task.id)
        self.tasks[task.id] = task
        self.pending_tasks.add(task.id)
        for dep in task.dependencies:
            self.task_dependencies[dep].append(task.id)

    def add_tasks(self, tasks: Sequence[Task]) -> None:
        for t in tasks:
            self.add_task(t)

    def param_size(self, param: str) -> float:
        c = self.param_cost
        if isinstance(c, (int, float)):
            return float(c)
        if callable(c):
            return float(c(param))
        return float(c.get(param, 0.5))

    # --------------------------------------------------------------- readiness
    def is_task_ready(self, task_id: str) -> bool:
        return all(dep in self.completed_tasks for dep in self.tasks[task_id].dependencies)

    def get_ready_tasks(self) -> List[Task]:
        source = self.pending_tasks if self.hash_order_compat else (t for t in self._insertion if t in self.pending_tasks)
        return [self.tasks[t] for t in source if self.is_task_ready(t)]

    # ------------------------------------------------------------ memory model
    def _load_cost(self, task: Task, node: Node) -> float:
        missing = task.params_needed - node.cached_params
        if isinstance(self.param_cost, (int, float)):
            return len(missing) * float(self.param_cost)
        return sum(self.param_size(p) for p in missing)

    def calculate_memory_requirement(self, task: Task, node: Node) -> float:
        return task.memory_required + self._load_cost(task, node)

    def can_fit_on_node(self, task: Task, node: Node) -> bool:
        return self.calculate_memory_requirement(task, node) <= node.available_memory

    def _event(self, action: str, node: Optional[str], item: str) -> None:
        self.events.append((self._round, action, node, item))

    def assign_task_to_node(self, task: Task, node: Node) -> bool:
        if self.calculate_memory_requirement(task, node) > node.available_memory:
            return False
        for p in sorted(task.params_needed - node.cached_params):
            node.cached_params.add(p)
            node.available_memory -= self.param_size(p)
            self.param_locations[p].add(node.id)
            self._event("LOAD", node.id, p)
        task.assigned_node = node.id
        node.running_tasks.append(task.id)
        node.available_memory -= task.memory_required
        self.pending_tasks.discard(task.id)
        node.last_used_params.extend(task.params_needed)
        self._event("RUN", node.id, task.id)
        # execution is instantaneous in the planning model (reference C6); the real
        # execution happens later in the executor, replaying self.events.
        self.complete_task(task.id)
        return True

    def complete_task(self, task_id: str) -> None:
        task = self.tasks.get(task_id)
        if task is None or not task.assigned_node:
            return
        node = self.nodes[task.assigned_node]
        task.completed = True
        self.completed_tasks.add(task_id)
        self.pending_tasks.discard(task_id)
        if task_id in node.running_tasks:
            node.running_tasks.remove(task_id)
        node.completed_tasks.append(task_id)
        node.available_memory += task.memory_required

    def fail_task(self, task_id: str) -> None:
        self.failed_tasks.add(task_id)
        self.pending_tasks.discard(task_id)
        self._event("FAIL", None, task_id)

    # ------------------------------------------------------------------ derived
    @property
    def orphaned_tasks(self) -> set:
        """Tasks neither completed nor failed (dependents of failed tasks)."""
        return set(self.tasks) - self.completed_tasks - self.failed_tasks

    def _is_fresh(self) -> bool:
        if self.completed_tasks or self.failed_tasks:
            return False
        return all(not n.cached_params and not n.completed_tasks and not n.running_tasks
                   and n.available_memory == n.total_memory for n in self.nodes.values())

    # ----------------------------------------------------------------- dispatch
    def schedule(self) -> Dict[str, List[str]]:
        use_native = (self.engine == "native" and self.native_policy is not None and not self.hash_order_compat
                      and self._is_fresh() and _native.available())
        if use_native:
            return self._schedule_native()
        return self._schedule_python()

    def _schedule_python(self) -> Dict[str, List[str]]:
        raise NotImplementedError

    # ---------------------------------------------------------- native engine
    def build_instance(self):
        core = _native.load()
        inst = core.Instance()
        ids = list(self._insertion)
        index = {t: i for i, t in enumerate(ids)}
        pnames: List[str] = []
        pindex: Dict[str, int] = {}
        params: List[List[int]] = []
        for t in ids:
            row = []
            for p in sorted(self.tasks[t].params_needed):
                if p not in pindex:
                    pindex[p] = len(pnames)
                    pnames.append(p)
                row.append(pindex[p])
            params.append(row)
        inst.task_ids = ids
        inst.mem = [float(self.tasks[t].memory_required) for t in ids]
        inst.compute = [float(self.tasks[t].compute_time) for t in ids]
        inst.deps = [[index.get(d, -1) for d in self.tasks[t].dependencies] for t in ids]
        inst.params = params
        inst.param_names = pnames
        inst.param_cost = [self.param_size(p) for p in pnames]
        node_list = list(self.nodes.values())
        inst.node_ids = [n.id for n in node_list]
        inst.node_mem = [float(n.total_memory) for n in node_list]
        inst.node_speed = [float(n.compute_speed) for n in node_list]
        inst.out_size = [float(getattr(self.tasks[t], "xfer_bytes", getattr(self.tasks[t], "out_bytes", 0)) or 0) / 1e9
                         for t in ids]
        self._configure_instance(inst)
        return inst, ids, pnames, node_list

    def _configure_instance(self, inst) -> None:
        pass

    def _schedule_native(self) -> Dict[str, List[str]]:
        core = _native.load()
        inst, ids, pnames, node_list = self.build_instance()
        res = core.run_policy(inst, self.native_policy)
        self._native_result = res
        self.rounds = res.rounds
        for i, tid in enumerate(ids):
            task = self.tasks[tid]
            n = res.assigned_node[i]
            if n >= 0:
                task.assigned_node = node_list[n].id
            if res.completed[i]:
                task.completed = True
                self.completed_tasks.add(tid)
            if res.failed[i]:
                self.failed_tasks.add(tid)
        self.pending_tasks = {t for t in ids if t not in self.completed_tasks and t not in self.failed_tasks}
        for n, node in enumerate(node_list):
            nr = res.nodes[n]
            node.available_memory = nr.available_memory
            node.cached_params = {pnames[p] for p in nr.cached}
            node.completed_tasks = [ids[t] for t in nr.completed]
            node.running_tasks = []
            node.last_used_params = deque((pnames[p] for p in nr.last_used), maxlen=10)
        names = {core.ACTION_RUN: "RUN", core.ACTION_LOAD: "LOAD", core.ACTION_EVICT: "EVICT", core.ACTION_FAIL: "FAIL"}
        self.events = []
        for rnd, act, n, item in res.events:
            a = names[act]
            node_id = node_list[n].id if n >= 0 else None
            item_id = ids[item] if a in ("RUN", "FAIL") else pnames[item]
            self.events.append((rnd, a, node_id, item_id))
            if a == "LOAD":
                self.param_locations[item_id]  # touch, like the reference's defaultdict
        for p in list(self.param_locations):
            self.param_locations[p] = {node.id for node in node_list if p in node.cached_params}
        self._after_native(res, ids, pnames)
        return {node_list[n].id: [ids[t] for t in res.schedule[n]] for n in res.node_first_use_order}

    def _after_native(self, res, ids, pnames) -> None:
        pass

    # ---------------------------------------------------------- python engine
    def _rounds(self, rank: Optional[Callable[[List[Task]], List[Task]]], choose: Callable[[Task], Optional[Node]],
                before_round: Optional[Callable[[], None]] = None,
                after_assign: Optional[Callable[[Task], None]] = None) -> Dict[str, List[str]]:
        """Round-synchronous loop shared by the four reference policies: the ready set is
        frozen at the start of a round (dependents of tasks placed in this round wait for
        the next one), at most 2|T| rounds, a round without progress fails everything
        still pending (reference C9-C15)."""
        placed: Dict[str, List[str]] = {}
        limit = 2 * len(self.tasks)
        it = 0
        while self.pending_tasks and it < limit:
            it += 1
            self._round = it
            if before_round is not None:
                before_round()
            ready = self.get_ready_tasks()
            if not ready:
                break
            if rank is not None:
                ready = rank(ready)
            progressed = False
            for task in ready:
                if task.id not in self.pending_tasks:
                    continue
                node = choose(task)
                if node is None:
                    self.fail_task(task.id)
                    continue
                if self.assign_task_to_node(task, node):
                    placed.setdefault(node.id, []).append(task.id)
                    progressed = True
                    if after_assign is not None:
                        after_assign(task)
            if not progressed:
                rest = list(self.pending_tasks) if self.hash_order_compat else \
                    [t for t in self._insertion if t in self.pending_tasks]
                for tid in rest:
                    self.fail_task(tid)
                break
        self.rounds = it
        return placed


def _topological(tasks: Dict[str, Task], order: Sequence[str]) -> List[str]:
    indeg = {t: 0 for t in order}
    kids = defaultdict(list)
    for t in order:
        for d in tasks[t].dependencies:
            if d in tasks:
                kids[d].append(t)
                indeg[t] += 1
    out = [t for t in order if indeg[t] == 0]
    i = 0
    while i < len(out):
        for k in kids[out[i]]:
            indeg[k] -= 1
            if indeg[k] == 0:
                out.append(k)
        i += 1
    seen = set(out)
    out.extend(t for t in order if t not in seen)
    return out


def task_depths(tasks: Dict[str, Task], order: Sequence[str]) -> Dict[str, int]:
    """Longest path (edge count) from a source, iteratively (reference C9 semantics)."""
    depth: Dict[str, int] = {}
    for t in _topological(tasks, order):
        deps = [d for d in tasks[t].dependencies if d in tasks]
        depth[t] = 0 if not tasks[t].dependencies else 1 + (max(depth.get(d, 0) for d in deps) if deps else 0)
    return depth


def bottom_levels(tasks: Dict[str, Task], order: Sequence[str], dependents: Mapping[str, List[str]]) -> Dict[str, float]:
    """b-level = own compute + max b-level over dependents (reference C11), iteratively."""
    bl: Dict[str, float] = {}
    for t in reversed(_topological(tasks, order)):
        kids = [d for d in dependents.get(t, []) if d in tasks]
        bl[t] = tasks[t].compute_time + max(bl.get(d, 0.0) for d in kids) if kids else tasks[t].compute_time
    return bl


class DFSScheduler(BaseScheduler):
    """Deepest-first; node with the most free memory (reference C9)."""

    native_policy = 0
    name = "DFS"

    def _schedule_python(self):
        depth = task_depths(self.tasks, self._insertion)

        def choose(task):
            best, most = None, -1
            for node in self.nodes.values():
                if self.can_fit_on_node(task, node) and node.available_memory > most:
                    best, most = node, node.available_memory
            return best

        return self._rounds(lambda r: sorted(r, key=lambda t: depth.get(t.id, 0), reverse=True), choose)


class GreedyScheduler(BaseScheduler):
    """Fewest parameter loads, then most free memory (reference C10). The chain-first
    variant described in the paper (Alg. 4) is available as ``identify_sequential_chains``
    for analysis, as in the reference it does not drive placement."""

    native_policy = 1
    name = "Greedy"

    def identify_sequential_chains(self) -> List[List[str]]:
        chains, seen = [], set()
        for start in (t for t in self._insertion if not self.tasks[t].dependencies):
            chain, cur = [], start
            while cur is not None and cur not in seen:
                chain.append(cur)
                seen.add(cur)
                nxt = self.task_dependencies.get(cur, [])
                cur = nxt[0] if len(nxt) == 1 and nxt[0] in self.tasks else None
            if len(chain) > 1:
                chains.append(chain)
        return chains

    def _schedule_python(self):
        def choose(task):
            best, fewest, roomiest = None, math.inf, 0
            for node in self.nodes.values():
                if not self.can_fit_on_node(task, node):
                    continue
                k = len(task.params_needed - node.cached_params)
                if k < fewest or (k == fewest and node.available_memory > roomiest):
                    best, fewest, roomiest = node, k, node.available_memory
            return best

        return self._rounds(None, choose)


class CriticalPathScheduler(BaseScheduler):
    """Longest bottom-level first; fastest fitting node (reference C11)."""

    native_policy = 2
    name = "Critical"

    def _schedule_python(self):
        bl = bottom_levels(self.tasks, self._insertion, self.task_dependencies)

        def choose(task):
            best, fastest = None, 0
            for node in self.nodes.values():
                if self.can_fit_on_node(task, node) and node.compute_speed > fastest:
                    best, fastest = node, node.compute_speed
            return best

        return self._rounds(lambda r: sorted(r, key=lambda t: bl.get(t.id, 0), reverse=True), choose)


class MRUScheduler(BaseScheduler):
    """Parameter-cache-aware placement with scored eviction ("MRU_spec", reference C12-C15).

    Node score = 20·|cached ∩ needed| + free memory (fits) or +5 (fits after eviction),
    minus 0.5·tasks completed on the node. Eviction victims are the cached parameters
    with the lowest ``10·uses + 100/(age+1) + 1000·[needed by a ready task]`` score. As in
    the reference, the eviction probe runs for real on every candidate node.
    """

    native_policy = 3
    name = "MRU_spec"

    def __init__(self, nodes, **kw):
        super().__init__(nodes, **kw)
        self.param_usage_count = defaultdict(int)
        self.param_last_used: Dict[str, int] = {}
        self.time_step = 0

    def calculate_eviction_score(self, param: str, node: Node) -> float:
        score = 0.0
        score += self.param_usage_count[param] * 10
        if param in self.param_last_used:
            score += 100.0 / (self.time_step - self.param_last_used[param] + 1)
        for tid in self.pending_tasks:
            if self.is_task_ready(tid) and param in self.tasks[tid].params_needed:
                score += 1000
        return score

    def evict_params_for_task(self, node: Node, task: Task) -> bool:
        shortage = self.calculate_memory_requirement(task, node) - node.available_memory
        if shortage <= 0:
            return True
        victims = sorted((self.calculate_eviction_score(p, node), p) for p in node.cached_params
                         if p not in task.params_needed)
        freed, gone = 0, []
        for _, p in victims:
            if freed >= shortage:
                break
            node.cached_params.remove(p)
            node.available_memory += self.param_size(p)
            self.param_locations[p].discard(node.id)
            freed += self.param_size(p)
            gone.append(p)
        if freed >= shortage:
            for p in gone:
                self._event("EVICT", node.id, p)
            return True
        for p in gone:  # roll back
            node.cached_params.add(p)
            node.available_memory -= self.param_size(p)
            self.param_locations[p].add(node.id)
        return False

    def _schedule_python(self):
        def bump():
            self.time_step += 1

        def urgency(task):
            return len([d for d in self.task_dependencies.get(task.id, []) if d in self.pending_tasks])

        def rank(ready):
            u = {t.id: urgency(t) for t in ready}
            return sorted(ready, key=lambda t: u[t.id], reverse=True)

        def choose(task):
            best, best_score = None, -float("inf")
            for node in self.nodes.values():
                score = 0.0
                score += len(task.params_needed & node.cached_params) * 20
                if self.can_fit_on_node(task, node):
                    score += node.available_memory
                elif self.evict_params_for_task(node, task):
                    score += 5
                else:
                    continue
                score -= len(node.completed_tasks) * 0.5
                if score > best_score:
                    best, best_score = node, score
            if best is not None and not self.can_fit_on_node(task, best):
                self.evict_params_for_task(best, task)
            return best

        def account(task):
            for p in task.params_needed:
                self.param_usage_count[p] += 1
                self.param_last_used[p] = self.time_step

        return self._rounds(rank, choose, before_round=bump, after_assign=account)

    def _after_native(self, res, ids, pnames):
        self.param_usage_count = defaultdict(int, {pnames[p]: c for p, c in enumerate(res.param_usage_count) if c})
        self.param_last_used = {pnames[p]: s for p, s in enumerate(res.param_last_used) if s >= 0}
        self.time_step = res.time_step


class EFTScheduler(BaseScheduler):
    """XGMI-EFT: transfer- and memory-aware earliest-finish-time placement (new).

    Priority = upward rank (compute + expected xGMI transfer to successors). Each ready
    task goes to the node minimising its finish time given the node's timeline, input
    arrivals (cross-GPU edges pay ``link_latency_s + bytes/link_bw``), parameter-cache
    fills on the node's copy engine (overlapped with compute) and the per-node memory cap.
    Eviction (``cyclic=True``, default): farthest next use first, counting the DAG's next
    repetition — the executor replays the plan every serving step, and for a layer chain
    under a cap this keeps the first layers resident across the step boundary so only the
    overflow is re-filled per step (least-recently-used order re-fills everything).
    ``refill_gb`` (pid -> GB a refill really moves, when the budget cost model differs, e.g.
    the reference's 0.5 GB per parameter): among eviction candidates the cheapest refill per
    unit of budget freed goes first, so under a flat cost the big groups stay resident.
    ``cyclic=False``: least useful first (not needed by a ready task, then oldest use). Sets
    ``start_time`` / ``finish_time`` per task (the planned, dependency-respecting timeline).

    Steady state (``steady=True``, default, with ``cyclic``): the executor replays the
    placement every step, so on N > 1 GPUs the cold pass above — which never finds an empty
    GPU better, every parameter being loaded once anyway — would leave one GPU re-filling the
    model's overflow every step while the others idle. When the cold pass re-fills anything,
    the native core also plans the repeating step (csrc/core/partition.h): a min-max pipeline
    partition of the DAG's topological order over the GPUs, stage busy = kernels
    (``real_time``: seconds per task, default ``compute_time``) + re-filled groups over the
    GPU's own host link + p2p edges; consecutive steps pipeline through the stages, so the
    step period is the busiest stage. The partition is kept when its modelled period is
    >= 2 % shorter (``cold_period`` / ``steady_period`` / ``partitioned`` / ``stages``).
    This is the reference's one-DAG-over-N-capped-nodes experiment
    (/root/reference/simulation.py:161-192, 375-376) planned for execution.
    """

    native_policy = 4
    name = "EFT"

    def __init__(self, nodes, *, link_bw_gbps: float = 153.0, link_latency_s: float = 5e-6,
                 load_bw_gbps: float = 50.0, cyclic: bool = True, refill_gb: Optional[Dict[str, float]] = None,
                 real_time: Optional[Dict[str, float]] = None, steady: bool = True, **kw):
        super().__init__(nodes, **kw)
        self.cyclic = cyclic
        self.steady = steady
        self.refill_gb = refill_gb
        self.real_time = real_time
        self.cold_period = self.steady_period = 0.0
        self.partitioned = False
        self.stages: List[Dict] = []
        self.link_bw_gbps = link_bw_gbps
        self.link_latency_s = link_latency_s
        self.load_bw_gbps = load_bw_gbps
        self.start_time: Dict[str, float] = {}
        self.finish_time: Dict[str, float] = {}

    def _configure_instance(self, inst) -> None:
        inst.link_bw = float(self.link_bw_gbps)
        inst.link_lat = float(self.link_latency_s)
        inst.load_bw = float(self.load_bw_gbps)
        inst.cyclic = bool(self.cyclic)
        inst.steady = bool(self.steady)
        if self.real_time is not None:
            inst.real_time = [float(self.real_time.get(t, self.tasks[t].compute_time)) for t in inst.task_ids]
        if self.refill_gb is not None:
            inst.param_refill = [float(self.refill_gb.get(p, self.param_size(p))) for p in inst.param_names]

    def _after_native(self, res, ids, pnames):
        self.start_time = {ids[i]: s for i, s in enumerate(res.start_time) if res.completed[i]}
        self.finish_time = {ids[i]: f for i, f in enumerate(res.finish_time) if res.completed[i]}
        self.cold_period, self.steady_period = float(res.cold_period), float(res.steady_period)
        self.partitioned = bool(res.partitioned)
        nids = list(self.nodes)
        self.stages = [{"node": nids[n], "busy_s": b, "refill_gb": g}
                       for n, b, g in zip(res.stage_node, res.stage_busy, res.stage_refill_gb)]

    def _schedule_python(self):
        raise RuntimeError("EFTScheduler requires the native core (distributed_llm_scheduler_amd._dlsched_core): "
                           f"{_native.error()}")


class GreedyChainScheduler(GreedyScheduler):
    """Chain-first greedy, as the paper describes it (PDF p.6 Alg. 4; the reference keeps
    ``identify_sequential_chains`` as dead code, schedulers.py:213-242).

    Phase 1: every sequential chain (from a source, following single dependents whose only
    dependency is the previous link) goes, in order, to the node with the most available
    memory at the time the chain is considered, until a link does not fit. Phase 2: the
    remaining tasks run through the round loop; each picks, among nodes it fits on, the
    one caching most of its parameters (ties: most available memory).
    """

    native_policy = None  # python engine only
    name = "Greedy_chain"

    def identify_sequential_chains(self) -> List[List[str]]:
        chains, seen = [], set()
        for start in (t for t in self._insertion if not self.tasks[t].dependencies):
            chain, cur = [], start
            while cur is not None and cur not in seen:
                chain.append(cur)
                seen.add(cur)
                nxt = self.task_dependencies.get(cur, [])
                cur = nxt[0] if (len(nxt) == 1 and nxt[0] in self.tasks
                                 and list(self.tasks[nxt[0]].dependencies) == [chain[-1]]) else None
            if len(chain) > 1:
                chains.append(chain)
        return chains

    def _schedule_python(self):
        placed: Dict[str, List[str]] = {}
        for chain in self.identify_sequential_chains():
            node = max(self.nodes.values(), key=lambda n: n.available_memory)  # first wins ties
            for tid in chain:
                task = self.tasks[tid]
                if tid not in self.pending_tasks or not self.is_task_ready(tid) or not self.can_fit_on_node(task, node):
                    break
                if self.assign_task_to_node(task, node):
                    placed.setdefault(node.id, []).append(tid)

        def choose(task):
            best, key = None, None
            for node in self.nodes.values():
                if not self.can_fit_on_node(task, node):
                    continue
                k = (len(task.params_needed & node.cached_params), node.available_memory)
                if key is None or k > key:
                    best, key = node, k
            return best

        for nid, tids in self._rounds(None, choose).items():
            placed.setdefault(nid, []).extend(tids)
        return placed


class MRUPaperScheduler(MRUScheduler):
    """MRU exactly as the paper's Alg. 5 writes it (PDF p.16): node score
    ``20·|P∩C| + 0.1·A − 0.5·|completed|``, −10 when the task only fits after eviction, and
    parameters scoring ≥ 1000 (needed by a ready task) are never eviction candidates. The
    code's variant (``MRU_spec``) uses ``+A``, ``+5`` and no filter."""

    native_policy = None  # python engine only
    name = "MRU_paper"

    def evict_params_for_task(self, node: Node, task: Task) -> bool:
        shortage = self.calculate_memory_requirement(task, node) - node.available_memory
        if shortage <= 0:
            return True
        cands = []
        for p in node.cached_params:
            if p in task.params_needed:
                continue
            sc = self.calculate_eviction_score(p, node)
            if sc < 1000:
                cands.append((sc, p))
        freed, gone = 0, []
        for _, p in sorted(cands):
            if freed >= shortage:
                break
            node.cached_params.remove(p)
            node.available_memory += self.param_size(p)
            self.param_locations[p].discard(node.id)
            freed += self.param_size(p)
            gone.append(p)
        if freed >= shortage:
            for p in gone:
                self._event("EVICT", node.id, p)
            return True
        for p in gone:
            node.cached_params.add(p)
            node.available_memory -= self.param_size(p)
            self.param_locations[p].add(node.id)
        return False

    def _schedule_python(self):
        def bump():
            self.time_step += 1

        def rank(ready):
            u = {t.id: len([d for d in self.task_dependencies.get(t.id, []) if d in self.pending_tasks])
                 for t in ready}
            return sorted(ready, key=lambda t: u[t.id], reverse=True)

        def choose(task):
            best, best_score = None, -float("inf")
            for node in self.nodes.values():
                score = len(task.params_needed & node.cached_params) * 20 + node.available_memory * 0.1
                score -= len(node.completed_tasks) * 0.5
                if self.can_fit_on_node(task, node):
                    pass
                elif self.evict_params_for_task(node, task):
                    score -= 10
                else:
                    continue
                if score > best_score:
                    best, best_score = node, score
            if best is not None and not self.can_fit_on_node(task, best):
                self.evict_params_for_task(best, task)
            return best

        def account(task):
            for p in task.params_needed:
                self.param_usage_count[p] += 1
                self.param_last_used[p] = self.time_step

        return self._rounds(rank, choose, before_round=bump, after_assign=account)


#: name -> class, using the reference's evaluation names (simulation.py:570-575)
SCHEDULERS = {
    "DFS": DFSScheduler,
    "Greedy": GreedyScheduler,
    "Critical": CriticalPathScheduler,
    "MRU_spec": MRUScheduler,
}
ALL_SCHEDULERS = dict(SCHEDULERS, EFT=EFTScheduler, Greedy_chain=GreedyChainScheduler, MRU_paper=MRUPaperScheduler)


def get_scheduler(name: str) -> type:
    key = {"critical path": "Critical", "criticalpath": "Critical", "mru": "MRU_spec", "dfs": "DFS",
           "greedy": "Greedy", "eft": "EFT", "xgmi-eft": "EFT"}.get(name.lower(), name)
    return ALL_SCHEDULERS[key]
