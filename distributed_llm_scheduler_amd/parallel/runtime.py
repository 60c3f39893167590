"""Glue: model DAG -> scheduler placement -> per-rank programs -> executors.

``plan(...)`` is deterministic and runs identically on every rank (no communication is
needed to agree on the placement): the DAG builder, the native scheduler and the program
lowering are pure functions of their arguments.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from ..core import Node, get_scheduler
from ..core.task import Task
from ..models import registry
from ..models.params import ParamStore, group_layout
from .program import Program, build_programs


@dataclass
class Plan:
    model: str
    tasks: List[Task]
    groups: Dict
    cfg: object
    scheduler_name: str
    scheduler: object
    schedule: Dict[str, List[str]]
    placement: Dict[str, int]
    order: List[str]
    node_rank: Dict[str, int]
    programs: List[Program]
    param_bytes: Dict[str, int]
    world: int
    cap_gb: float
    stats: Dict = field(default_factory=dict)

    @property
    def completed(self) -> int:
        return len(self.scheduler.completed_tasks)

    @property
    def total(self) -> int:
        return len(self.tasks)


def plan(model: str = "gpt2", world: int = 1, scheduler: str = "EFT", cap_gb: float = 288.0, replicas: int = 1,
         batch: int = 1, seq: int = 512, cost_model: str = "bytes", fuse: bool = True,
         node_speeds: Optional[Sequence[float]] = None, link_bw_gbps: float = 153.0,
         placement: str = "scheduler", tp: int = 1) -> Plan:
    """Build the DAG of ``replicas`` requests of ``model``, place it on ``world`` GPUs with
    ``scheduler`` under a per-GPU cap of ``cap_gb`` and lower it to per-rank programs.

    ``placement``:
      * ``"scheduler"`` — the policy decides (default),
      * ``"replica"``   — request r on GPU r % world (plain data parallelism, a baseline),
      * ``"pipeline"``  — contiguous layer blocks per GPU, requests act as micro-batches
        (pipeline parallelism: each block boundary is a cross-GPU p2p edge),
      * ``"tensor"``    — with ``tp > 1``: shard k of every layer on GPU k % world, the
        shard-sum / residual / embedding / head nodes on GPU 0 (tensor parallelism).
    The fixed placements still go through the scheduler's memory accounting (tasks that
    do not fit fail exactly as in the policies).
    """
    tasks, groups, cfg = registry.build(model, batch=batch, seq=seq, replicas=replicas, cost_model=cost_model, tp=tp)
    param_bytes = {pid: group_layout(g)[0] for pid, g in groups.items()}
    nodes = [Node(f"gpu{r}", cap_gb, (node_speeds[r] if node_speeds else 1.0), device=r) for r in range(world)]
    node_rank = {n.id: r for r, n in enumerate(nodes)}
    cls = get_scheduler(scheduler)
    kw = {}
    if cost_model == "bytes":
        kw["param_cost"] = {pid: b / 1e9 for pid, b in param_bytes.items()}
    if cls.__name__ == "EFTScheduler":
        kw["link_bw_gbps"] = link_bw_gbps
    sched = cls([n.fresh() for n in nodes], **kw)
    for t in tasks:
        sched.add_task(t.clone())
    if placement == "scheduler":
        schedule = sched.schedule()
    elif placement in ("replica", "pipeline", "tensor"):
        schedule = _fixed_schedule(tasks, world, sched, placement, cfg)
    else:
        raise ValueError(f"unknown placement {placement!r}")
    place = {tid: node_rank[sched.tasks[tid].assigned_node] for tid in sched.completed_tasks}
    order = [item for _, act, _, item in sched.events if act == "RUN"]
    caps = {r: int(cap_gb * 1e9) for r in range(world)}
    programs = build_programs(tasks, place, order, world, param_bytes, caps, events=sched.events,
                              node_rank=node_rank, fuse=fuse)
    p = Plan(model, tasks, groups, cfg, cls.name if placement == "scheduler" else placement, sched, schedule, place, order, node_rank, programs, param_bytes,
             world, cap_gb)
    p.stats = plan_stats(p)
    return p


def _layer_of(tid: str, n_layer: int) -> int:
    """Pipeline position of a task: embedding -> -1, layer_i_* -> i, head -> n_layer."""
    base = tid.split("/")[-1]
    if base.startswith("layer_"):
        return int(base.split("_")[1])
    return -1 if base in ("embedding",) else n_layer


def _fixed_schedule(tasks: Sequence[Task], world: int, sched, mode: str, cfg) -> Dict[str, List[str]]:
    """Place without the policy: by replica (DP) or by contiguous layer blocks (PP).
    Tasks are committed in DAG order; memory is still accounted per node."""
    out: Dict[str, List[str]] = {}
    nodes = list(sched.nodes.values())
    L = cfg.n_layer
    for t in tasks:
        if mode == "replica":
            rep = int(t.id.split("/")[0][1:]) if "/" in t.id else 0
            r = rep % world
        elif mode == "tensor":
            sfx = t.id.rsplit(".", 1)[-1] if "." in t.id.split("/")[-1] else ""
            r = int(sfx[2:]) % world if sfx.startswith("tp") and sfx[2:].isdigit() else 0
        else:
            layer = min(max(_layer_of(t.id, L), 0), L - 1)
            r = min(layer * world // L, world - 1)
        node = nodes[r]
        if any(d in sched.failed_tasks or d not in sched.completed_tasks for d in t.dependencies) \
                or not sched.assign_task_to_node(sched.tasks[t.id], node):
            sched.fail_task(t.id)
            continue
        out.setdefault(node.id, []).append(t.id)
    return out


def plan_stats(p: Plan) -> Dict:
    cross = 0
    cross_bytes = 0
    tmap = {t.id: t for t in p.tasks}
    for tid, r in p.placement.items():
        for d in tmap[tid].dependencies:
            if d in p.placement and p.placement[d] != r:
                cross += 1
                cross_bytes += tmap[d].out_bytes
    return {
        "tasks_total": len(p.tasks),
        "tasks_completed": len(p.scheduler.completed_tasks),
        "tasks_failed": len(p.scheduler.failed_tasks),
        "tasks_orphaned": len(p.scheduler.orphaned_tasks),
        "cross_gpu_edges": cross,
        "cross_gpu_bytes": cross_bytes,
        "kernels_per_rank": [pr.n_kernels for pr in p.programs],
        "param_peak_gb_per_rank": [pr.param_peak_bytes / 1e9 for pr in p.programs],
        "act_arena_gb_per_rank": [pr.act_arena_bytes / 1e9 for pr in p.programs],
        "tasks_per_rank": [sum(1 for r in p.placement.values() if r == k) for k in range(p.world)],
    }


def make_store(p: Plan, seed: int = 0, device_init: bool = False) -> ParamStore:
    return ParamStore(p.groups, seed=seed, device_init=device_init)


def make_executor(p: Plan, rank: int, device, store: Optional[ParamStore] = None, pg=None, use_graph: bool = True,
                  trace: bool = False):
    from .executor import DAGExecutor

    return DAGExecutor(p.tasks, p.programs[rank], store or make_store(p), device, model_cfg=p.cfg,
                       use_graph=use_graph, pg=pg, trace=trace)
