"""Glue: model DAG -> scheduler placement -> per-rank programs -> executors.

``plan(...)`` is deterministic and runs identically on every rank (no communication is
needed to agree on the placement): the DAG builder, the native scheduler and the program
lowering are pure functions of their arguments.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from ..core import Node, get_scheduler
from ..core.task import Task
from ..models import registry
from ..models.params import ParamStore, group_layout
from .program import Program, build_programs, build_steady_programs, plan_peer_fills, steady_fill_bytes


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
    args: Dict = field(default_factory=dict)  # plan() arguments (checkpoint / replan)

    @property
    def completed(self) -> int:
        return len(self.scheduler.completed_tasks)

    @property
    def total(self) -> int:
        return len(self.tasks)


def plan(model: str = "gpt2", world: int = 1, scheduler: str = "EFT", cap_gb: float = 288.0, replicas: int = 1,
         batch: int = 1, seq: int = 512, cost_model: str = "bytes", fuse: bool = True,
         node_speeds: Optional[Sequence[float]] = None, link_bw_gbps: float = 153.0,
         placement: str = "scheduler", tp: int = 1, resume: Optional[str] = None, sp: int = 1,
         residency: Optional[str] = None) -> Plan:
    """Build the DAG of ``replicas`` requests of ``model``, place it on ``world`` GPUs with
    ``scheduler`` under a per-GPU cap of ``cap_gb`` (one value, or one per GPU — the
    reference's heterogeneous node splits) and lower it to per-rank programs.

    ``placement``:
      * ``"scheduler"`` — the policy decides (default),
      * ``"replica"``   — request r on GPU r % world (plain data parallelism, a baseline),
      * ``"pipeline"``  — contiguous layer blocks per GPU, requests act as micro-batches
        (pipeline parallelism: each block boundary is a cross-GPU p2p edge),
      * ``"tensor"``    — with ``tp > 1``: shard k of every layer on GPU k % world, the
        shard-sum / residual / embedding / head nodes on GPU 0 (tensor parallelism).
      * ``"sequence"``  — with ``sp > 1``: sequence chunk c of every node on GPU c % world
        (context parallelism; the K/V edges between chunks are the cross-GPU transfers).
      * ``"expert"``    — MoE models: expert e of every layer on GPU e % world, everything
        else of request r on its home GPU r % world (expert parallelism: the router ->
        expert edges carry each expert's routed token rows, the expert -> combine edges its
        compact outputs).
    The fixed placements still go through the scheduler's memory accounting (tasks that
    do not fit fail exactly as in the policies).

    ``residency`` (default ``$DLS_RESIDENCY`` or ``"auto"``): how parameter residency of the
    repeating step is lowered — ``"trace"`` replays the policy's LOAD/EVICT trace (cold or
    warm-started, program.build_steady_programs); ``"auto"`` additionally offers a policy
    whose memory model is the repeating step (EFT) the planned keep set
    (program.plan_keep_sets) and keeps whichever re-fills fewer bytes per step.

    ``resume``: path of a placement saved by :func:`save_plan` — the saved decision (task
    order per GPU and the LOAD/EVICT trace) is reused instead of re-running the policy; the
    DAG is rebuilt from the saved arguments, which must match this call's.
    """
    caps_gb = [float(c) for c in cap_gb] if isinstance(cap_gb, (list, tuple)) else [float(cap_gb)] * world
    if len(caps_gb) != world:
        raise ValueError(f"{len(caps_gb)} per-GPU caps for world {world}")
    if isinstance(cap_gb, (list, tuple)):
        cap_gb = list(caps_gb)
    args = dict(model=model, world=world, scheduler=scheduler, cap_gb=cap_gb, replicas=replicas, batch=batch,
                seq=seq, cost_model=cost_model, fuse=fuse, node_speeds=list(node_speeds) if node_speeds else None,
                link_bw_gbps=link_bw_gbps, placement=placement, tp=tp)
    if sp > 1:
        args["sp"] = sp
    tasks, groups, cfg = registry.build(model, batch=batch, seq=seq, replicas=replicas, cost_model=cost_model, tp=tp,
                                        sp=sp)
    param_bytes = {pid: group_layout(g)[0] for pid, g in groups.items()}
    nodes = [Node(f"gpu{r}", caps_gb[r], (node_speeds[r] if node_speeds else 1.0), device=r) for r in range(world)]
    node_rank = {n.id: r for r, n in enumerate(nodes)}
    cls = get_scheduler(scheduler)
    kw = {}
    if cost_model == "bytes":
        kw["param_cost"] = {pid: b / 1e9 for pid, b in param_bytes.items()}
    if cls.__name__ == "EFTScheduler":
        kw["link_bw_gbps"] = link_bw_gbps
        kw["refill_gb"] = {pid: b / 1e9 for pid, b in param_bytes.items()}  # what a refill really moves
    sched = cls([n.fresh() for n in nodes], **kw)
    for t in tasks:
        sched.add_task(t.clone())
    if resume is not None:
        sched, schedule = _resume(resume, args, sched)
    elif placement == "scheduler":
        schedule = sched.schedule()
    elif placement in ("replica", "pipeline", "tensor", "sequence", "expert"):
        schedule = _fixed_schedule(tasks, world, sched, placement, cfg)
    else:
        raise ValueError(f"unknown placement {placement!r}")
    place = {tid: node_rank[sched.tasks[tid].assigned_node] for tid in sched.completed_tasks}
    order = [item for _, act, _, item in sched.events if act == "RUN"]
    caps = {r: int(caps_gb[r] * 1e9) for r in range(world)}
    residency = residency or os.environ.get("DLS_RESIDENCY", "auto")
    if residency not in ("auto", "trace"):
        raise ValueError(f"unknown residency {residency!r}")
    planned = None
    if residency == "auto" and getattr(sched, "cyclic", False):
        # EFT's memory model is the repeating step: its residency may be the planned keep set
        # (program.plan_keep_sets) under the same budget the policy accounted: the node cap
        # minus the largest activation requirement among the node's tasks
        tmem = {t.id: t.memory_required for t in tasks}
        budget = {r: caps_gb[r] - max([tmem[tid] for tid, rr in place.items() if rr == r] or [0.0])
                  for r in range(world)}
        planned = (budget, {pid: sched.param_size(pid) for pid in param_bytes})
    prefetch = os.environ.get("DLS_PREFETCH", "auto")  # executor.PREFETCH
    programs = build_steady_programs(tasks, place, order, world, param_bytes, caps, events=sched.events,
                                     node_rank=node_rank, fuse=fuse, planned=planned,
                                     lookahead=0 if prefetch == "0" else 1, force_ahead=prefetch == "1")
    if world > 1 and os.environ.get("DLS_PEER_FILL", "1") != "0":
        plan_peer_fills(programs, tasks, param_bytes)  # refills from a peer's HBM over xGMI
    name = cls.name if placement == "scheduler" else placement
    p = Plan(model, tasks, groups, cfg, name, sched, schedule, place, order, node_rank, programs, param_bytes,
             world, cap_gb, args=args)
    p.stats = plan_stats(p)
    return p


_PLAN_FORMAT = "dlsched-plan/1"


def save_plan(p: Plan, path: str) -> None:
    """Checkpoint a placement: the plan() arguments, the per-GPU task order and the
    scheduler's action trace (RUN / LOAD / EVICT / FAIL). Resume with ``plan(resume=path)``."""
    s = p.scheduler
    doc = {"format": _PLAN_FORMAT, "args": p.args, "scheduler": p.scheduler_name, "schedule": p.schedule,
           "events": [list(e) for e in s.events], "failed": sorted(s.failed_tasks),
           "stats": {k: v for k, v in p.stats.items() if isinstance(v, (int, float, list))}}
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)


class _ResumedSchedule:
    """Scheduler-shaped view of a saved decision (what build_programs / Plan consume)."""

    def __init__(self, sched, doc):
        self.tasks = sched.tasks
        self.nodes = sched.nodes
        self.events = [tuple(e) for e in doc["events"]]
        self.failed_tasks = set(doc.get("failed", []))
        self.completed_tasks = set()
        self.orphaned_tasks = set()
        for _, act, node, item in self.events:
            if act == "RUN":
                if item not in self.tasks:
                    raise ValueError(f"saved placement runs unknown task {item!r}")
                self.tasks[item].assigned_node = node
                self.completed_tasks.add(item)
        self.orphaned_tasks = set(self.tasks) - self.completed_tasks - self.failed_tasks


def _resume(path: str, args: Dict, sched):
    with open(path) as f:
        doc = json.load(f)
    if doc.get("format") != _PLAN_FORMAT:
        raise ValueError(f"{path}: not a saved plan")
    saved = dict(doc["args"])
    mismatch = {k: (saved.get(k), v) for k, v in args.items() if k not in ("fuse",) and saved.get(k) != v}
    if mismatch:
        raise ValueError(f"saved plan was made with different arguments: {mismatch}")
    return _ResumedSchedule(sched, doc), {k: list(v) for k, v in doc["schedule"].items()}


def replan(p: Plan, lost_ranks: Sequence[int], **overrides) -> Plan:
    """Device loss: re-place the whole DAG on the surviving GPUs (ranks renumbered densely,
    speeds kept). The SURVEY §5 "device-loss injection -> re-plan onto survivors" path; the
    executor side is :func:`make_executor` on the new plan's programs."""
    lost = set(lost_ranks)
    keep = [r for r in range(p.world) if r not in lost]
    if not keep:
        raise RuntimeError("no surviving devices")
    a = dict(p.args)
    a.update(world=len(keep))
    if a.get("node_speeds"):
        a["node_speeds"] = [a["node_speeds"][r] for r in keep]
    if isinstance(a.get("cap_gb"), list):
        a["cap_gb"] = [a["cap_gb"][r] for r in keep]
    a.update(overrides)
    return plan(**a)


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
        if mode in ("replica", "expert"):
            rep = int(t.id.split("/")[0][1:]) if "/" in t.id else 0
            r = rep % world
            if mode == "expert" and t.op is not None and t.op.kind == "moe_expert":
                r = t.op.attrs["expert"] % world
        elif mode in ("tensor", "sequence"):
            tag = "tp" if mode == "tensor" else "sp"
            sfx = t.id.rsplit(".", 1)[-1] if "." in t.id.split("/")[-1] else ""
            r = int(sfx[2:]) % world if sfx.startswith(tag) and sfx[2:].isdigit() else 0
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
                cross_bytes += tmap[d].xfer_bytes
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
        # parameter bytes re-filled per steady-state step (evict/reload traffic of the plan)
        "refill_gb_per_step_per_rank": [steady_fill_bytes(pr, p.param_bytes) / 1e9 for pr in p.programs],
        # of which received from a peer GPU's arena over xGMI (RCCL p2p) instead of the host
        "peer_fill_gb_per_step_per_rank": [sum(int(p.param_bytes.get(i.param, 0)) for i in pr.instrs
                                               if i.op == "load" and i.peer >= 0) / 1e9 for pr in p.programs],
        "tasks_per_rank": [sum(1 for r in p.placement.values() if r == k) for k in range(p.world)],
    }


def make_store(p: Plan, seed: int = 0, device_init: bool = False) -> ParamStore:
    return ParamStore(p.groups, seed=seed, device_init=device_init)


def device_init_ok(p: Plan, rank: int) -> bool:
    """Can rank's weights be random-initialised straight into HBM? Only when its program
    re-fills nothing in the steady state: every refill of an evicted/overwritten group must
    be a real host->HBM copy (a measured cost, and capturable in a hipGraph)."""
    return steady_fill_bytes(p.programs[rank], p.param_bytes) == 0


def make_executor(p: Plan, rank: int, device, store: Optional[ParamStore] = None, pg=None, use_graph: bool = True,
                  trace: bool = False, debug: bool = False, autotune: bool = True):
    """``debug=True``: validate every rank's program first (parallel/validate.py) and run the
    executor with arena canaries and output finiteness checks. ``autotune=False``: GEMM shapes
    missing from the tuning table run the kernel's heuristic config instead of being tuned first."""
    from .executor import DAGExecutor

    if debug:
        from .validate import check_plan

        errs = check_plan(p)
        if errs:
            raise RuntimeError("invalid plan:\n  " + "\n  ".join(errs[:20]))
    # per-model GEMM choices by the canonical preset name (aliases such as "mixtral" resolve to it)
    return DAGExecutor(p.tasks, p.programs[rank], store or make_store(p), device, model_cfg=p.cfg,
                       use_graph=use_graph, pg=pg, trace=trace, debug=debug, model_name=p.cfg.name, autotune=autotune)
