"""Glue: model DAG -> scheduler placement -> per-rank programs -> executors.

``plan(...)`` is deterministic and runs identically on every rank (no communication is
needed to agree on the placement): the DAG builder, the native scheduler and the program
lowering are pure functions of their arguments.
"""
from __future__ import annotations

import json
import math
import os
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

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
    # merged micro-batches (merge_mb > 1): request prefix "r{k}/" -> (merged prefix, batch
    # rows lo, hi) and merged token input -> the requests' token inputs, in row order
    requests: Dict = field(default_factory=dict)
    input_parts: Dict = field(default_factory=dict)

    def owner(self, tid: str) -> Optional[int]:
        """Rank holding task ``tid``'s output (a merged request resolves to its group)."""
        if tid in self.placement:
            return self.placement[tid]
        if "/" in tid and self.requests:
            rid, base = tid.split("/", 1)
            m = self.requests.get(rid + "/")
            return self.placement.get(m[0] + base) if m else None
        return None

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
         residency: Optional[str] = None, merge_mb: int = 1) -> Plan:
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

    ``merge_mb`` = k > 1: the ``replicas`` requests are micro-batches of one batch, merged k at
    a time into one request of batch k x ``batch`` BEFORE placement (a DAG transform: every
    node of k co-located micro-batches becomes ONE node over k x the rows — one M = k x 512
    GEMM instead of k M = 512 launches, one p2p edge of k x the bytes instead of k). Every
    request keeps its own token ids and its own rows of the merged outputs
    (``Plan.requests``, ``DAGExecutor.output("r{k}/...")``).

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
    requests, input_parts = {}, {}
    n_req, mb_batch = replicas, batch
    if merge_mb > 1:
        if replicas % merge_mb:
            raise ValueError(f"merge_mb={merge_mb} must divide replicas={replicas}")
        args["merge_mb"] = merge_mb
        n_req, mb_batch = replicas // merge_mb, batch * merge_mb
        for g in range(n_req):
            pre = f"r{g}/" if n_req > 1 else ""
            members = list(range(g * merge_mb, (g + 1) * merge_mb))
            input_parts[f"{pre}@tokens"] = [f"r{k}/@tokens" if replicas > 1 else "@tokens" for k in members]
            for j, k in enumerate(members):
                requests[f"r{k}/"] = (pre, j * batch, (j + 1) * batch)
    tasks, groups, cfg = registry.build(model, batch=mb_batch, seq=seq, replicas=n_req, cost_model=cost_model, tp=tp,
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
        # the steady-state model needs real seconds, not abstract constants: the per-task kernel
        # times measured on an MI355X (ops/task_times.json, as the pipeline balancer uses) where
        # the table has the model, the roofline estimate elsewhere
        measured = measured_task_times(task_times_key(cfg.name, seq, mb_batch))
        if measured or cost_model != "bytes":
            kw["real_time"] = {t.id: measured.get(_base_id(t.id), real_time_s(t, param_bytes)) for t in tasks}
    sched = cls([n.fresh() for n in nodes], **kw)
    for t in tasks:
        sched.add_task(t.clone())
    if resume is not None:
        sched, schedule = _resume(resume, args, sched)
    elif placement == "scheduler":
        schedule = sched.schedule()
    elif placement in ("replica", "pipeline", "tensor", "sequence", "expert"):
        stage_of = None
        if placement == "pipeline" and world > 1 and os.environ.get("DLS_PIPELINE_STAGES", "balanced") != "layers":
            stage_of = pipeline_stages(tasks, world, param_bytes, caps_gb, node_speeds, n_req,
                                       task_times_key(cfg.name, seq, mb_batch))
        order_in = tasks
        if placement == "expert" and world > 1 and n_req > 1:
            order_in = _interleave_requests(tasks)  # every GPU steps through the layers together
        schedule = _fixed_schedule(order_in, world, sched, placement, cfg, stage_of)
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
             world, cap_gb, args=args, requests=requests, input_parts=input_parts)
    p.stats = plan_stats(p)
    return p


def real_time_s(t: Task, param_bytes: Dict[str, int]) -> float:
    """Roofline seconds of one task on one MI355X (the ``bytes`` cost model's estimate:
    models/gpt2._roofline), whatever cost model the task's ``compute_time`` is in."""
    from ..models.gpt2 import _roofline

    moved = float(getattr(t, "out_bytes", 0) or 0) + sum(float(param_bytes.get(p, 0)) for p in t.params_needed)
    return _roofline(float(getattr(t, "flops", 0.0) or 0.0), moved)


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


def _base_id(tid: str) -> str:
    return tid.split("/", 1)[1] if "/" in tid and tid[0] == "r" and tid.split("/", 1)[0][1:].isdigit() else tid


def pipeline_stages(tasks: Sequence[Task], world: int, param_bytes: Dict[str, int], caps_gb: Sequence[float],
                    node_speeds: Optional[Sequence[float]], replicas: int, model: str) -> Optional[Dict[str, int]]:
    """Pipeline stages balanced by kernel time (the VERDICT r4 item: layer-count blocks left
    half the stages idle half the time): a min-max partition of ONE request's DAG over the GPUs
    (the native steady-state partition, csrc/core/partition.h), every micro-batch's task on
    its base task's GPU. A stage's cost per step = its tasks' kernel time x the micro-batches +
    the p2p edges it sends and receives; cut points are the DAG's clean boundaries (the residual
    stream alone: attention / MLP half-layers), so no fused kernel pair is split. Kernel times:
    the measured per-task table (``ops/task_times.json``, written by
    ``benchmarks/measure_task_times.py`` on an MI355X) when it has the model, else the roofline
    (:func:`real_time_s`). Returns base task id -> GPU, or None (no native core / infeasible:
    the caller keeps layer-count blocks)."""
    from ..core import native as _native

    try:
        core = _native.load()
    except Exception:  # noqa: BLE001 — the layer-count split still works
        return None
    base = [t for t in tasks if _base_id(t.id) == t.id or t.id.startswith("r0/")]
    ids = [_base_id(t.id) for t in base]
    index = {tid: i for i, tid in enumerate(ids)}
    measured = measured_task_times(model)
    R = max(int(replicas), 1)
    pn, pidx, prow = [], {}, []
    for t in base:
        row = []
        for p in sorted(t.params_needed):
            if p not in pidx:
                pidx[p] = len(pn)
                pn.append(p)
            row.append(pidx[p])
        prow.append(row)
    inst = core.Instance()
    inst.task_ids = ids
    inst.mem = [float(t.out_bytes) * R / 1e9 for t in base]
    times = [measured.get(i, real_time_s(t, param_bytes)) if measured else real_time_s(t, param_bytes)
             for i, t in zip(ids, base)]
    inst.compute = [v * R for v in times]
    inst.real_time = list(inst.compute)
    inst.deps = [[index.get(_base_id(d), -1) for d in t.dependencies] for t in base]
    inst.params = prow
    inst.param_names = pn
    inst.param_cost = [param_bytes.get(p, 0) / 1e9 for p in pn]
    inst.param_refill = list(inst.param_cost)
    inst.node_ids = [f"gpu{r}" for r in range(world)]
    inst.node_mem = [float(c) for c in caps_gb]
    inst.node_speed = [float(v) for v in node_speeds] if node_speeds else [1.0] * world
    inst.out_size = [float(t.out_bytes) * R / 1e9 for t in base]
    # fused kernel chains of the lowering (program._fusion): a stage cut never splits one
    from .program import _consumers, _fusion
    tmap = {t.id: t for t in base}
    one = {t.id: 0 for t in base}
    order = [t.id for t in base]
    fused_into, _ = _fusion(tmap, one, order, _consumers(tmap, one, order), {t: i for i, t in enumerate(order)}, True)
    inst.fuse_into = [index[_base_id(fused_into[t.id])] if t.id in fused_into else -1 for t in base]
    part = core.steady_partition(inst, world, world)
    if not part.feasible:
        return None
    return {ids[i]: int(n) for i, n in enumerate(part.node_of_task) if n >= 0}


_TASK_TIMES: Dict[str, Dict[str, float]] = {}


def task_times_key(model: str, seq: int, batch: int) -> str:
    return f"{model}/s{seq}b{batch}"


def measured_task_times(key: str) -> Dict[str, float]:
    """Per-task kernel seconds measured on an MI355X (base task ids; a fused kernel group's
    time split over its tasks) for ``key`` = :func:`task_times_key`, from
    ``ops/task_times.json``; a batch the table lacks is scaled from batch 1 (an upper bound:
    bigger GEMMs run closer to peak); {} if absent."""
    if not _TASK_TIMES:
        path = os.environ.get("DLS_TASK_TIMES") or os.path.join(os.path.dirname(__file__), "..", "ops",
                                                                  "task_times.json")
        try:
            with open(path) as f:
                _TASK_TIMES.update(json.load(f))
        except (OSError, ValueError):
            _TASK_TIMES["__none__"] = {}
    if key in _TASK_TIMES:
        return dict(_TASK_TIMES[key])
    head, _, b = key.rpartition("b")
    if b.isdigit() and int(b) > 1 and (head + "b1") in _TASK_TIMES:
        return {t: v * int(b) for t, v in _TASK_TIMES[head + "b1"].items()}
    return {}


def _interleave_requests(tasks: Sequence[Task]) -> List[Task]:
    """Layer-major order of replicated requests (identical DAGs, ids ``r{k}/...``): the i-th
    task of every request before the (i+1)-th of any. With data-parallel attention and expert
    parallelism each GPU is home to one request and hosts experts of all of them; request-major
    order would run the requests one after another across the whole job (each GPU's experts
    serve request 0's 32 layers before its own request starts), whereas here every GPU works on
    the same layer, and one layer's expert nodes of all requests sit next to each other in its
    program — the co-run span (program.plan_coruns) that streams each expert's weights once."""
    seen: Dict[str, int] = defaultdict(int)
    keyed = []
    for n, t in enumerate(tasks):
        rep = t.id.split("/", 1)[0] if "/" in t.id else ""
        keyed.append((seen[rep], n, t))
        seen[rep] += 1
    return [t for _, _, t in sorted(keyed, key=lambda x: (x[0], x[1]))]


def _fixed_schedule(tasks: Sequence[Task], world: int, sched, mode: str, cfg,
                    stage_of: Optional[Dict[str, int]] = None) -> Dict[str, List[str]]:
    """Place without the policy: by replica (DP) or by contiguous pipeline stages (PP:
    ``stage_of`` base task -> GPU from :func:`pipeline_stages`, else layer-count blocks).
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
        elif stage_of is not None and _base_id(t.id) in stage_of:
            r = stage_of[_base_id(t.id)]
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
        # distinct (producer, consumer GPU) transfers: what the p2p edges really move
        "cross_gpu_transfers": len({(d, r) for tid, r in p.placement.items() for d in tmap[tid].dependencies
                                    if d in p.placement and p.placement[d] != r}),
        # what the same transfers move when expert-parallel edges carry routed rows only (the
        # device transport, DAGExecutor._plan_routed_edges): expected M*k/E rows per expert
        "cross_gpu_bytes_routed": _routed_cross_bytes(p, tmap),
        # what the programs' p2p sends move per step on the RCCL transport: whole buffers, except
        # expert-parallel capacity edges (program.plan_ep_capacity: EP_CAPACITY x the expected
        # routed rows, fixed-size messages)
        "cross_gpu_bytes_rccl": _rccl_send_bytes(p, tmap),
        **_steady_stats(p.scheduler),
    }


def _rccl_send_bytes(p: Plan, tmap) -> int:
    total = 0
    for pr in p.programs:
        for i in pr.instrs:
            if i.op != "send":
                continue
            t = tmap[i.task]
            if i.rows and t.op is not None and t.op.out_shape:
                total += int(t.xfer_bytes * i.rows / math.prod(t.op.out_shape[:-1]))
            else:
                total += t.xfer_bytes
    return total


def _routed_cross_bytes(p: Plan, tmap) -> int:
    """Cross-GPU bytes per step with routed-row expert edges: a hidden state sent to a GPU whose
    consumers there are experts moves the rows routed to those experts (expected M*k/E per
    expert), an expert's output its routed rows; every other transfer its whole buffer."""
    total = 0
    users_at: Dict[Tuple[str, int], List[Task]] = {}
    for tid, r in p.placement.items():
        for d in tmap[tid].dependencies:
            if d in p.placement and p.placement[d] != r:
                users_at.setdefault((d, r), []).append(tmap[tid])
    for (d, r), users in users_at.items():
        t = tmap[d]
        exp_users = [u for u in users if u.op is not None and u.op.kind == "moe_expert" and u.op.inputs[0] == d]
        if users and len(exp_users) == len(users):
            a = exp_users[0].op.attrs
            total += int(t.xfer_bytes * a["top_k"] * len(exp_users) / a["n_experts"])
        elif t.op is not None and t.op.kind == "moe_expert":
            total += int(t.xfer_bytes * t.op.attrs["top_k"] / t.op.attrs["n_experts"])
        else:
            total += t.xfer_bytes
    return total


def _steady_stats(s) -> Dict:
    """EFT's steady-state model (csrc/core/partition.h): modelled step period of its cold pass
    and of the placement it returned, and whether the pipeline partition replaced the cold pass."""
    if not hasattr(s, "steady_period") or not getattr(s, "cold_period", 0.0):
        return {}
    return {"eft_partitioned": bool(s.partitioned), "modelled_period_ms": round(s.steady_period * 1e3, 4),
            "modelled_cold_period_ms": round(s.cold_period * 1e3, 4),
            "stages": [{"node": st["node"], "busy_ms": round(st["busy_s"] * 1e3, 4),
                        "refill_gb": round(st["refill_gb"], 6)} for st in s.stages]}


def torch_device_type(device) -> str:
    import torch

    return torch.device(device).type


def ep_widen_on_overflow(ex, pg=None) -> bool:
    """After a step of an expert-parallel job (one process per rank): did any rank's capacity
    edge overflow? (one all-reduce; a host read of this rank's flags). If so every rank widens
    the groups IT saw overflow (both ranks of a group see the same routing counts) and the
    caller re-runs the step — and re-captures, if it captured — then calls this again: a
    corrected layer can change a later layer's routing, so repeat until it returns False."""
    import torch
    import torch.distributed as dist

    mine = ex.ep_overflow()
    flag = torch.tensor([1 if mine else 0], dtype=torch.int32,
                        device=ex.device if (ex.gpu and pg is not None and dist.get_backend(pg) == "nccl") else "cpu")
    if pg is not None:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=pg)
    if not int(flag.item()):
        return False
    ex.widen_ep(mine)
    return True


def make_store(p: Plan, seed: int = 0, device_init: bool = False) -> ParamStore:
    return ParamStore(p.groups, seed=seed, device_init=device_init)


def device_init_ok(p: Plan, rank: int) -> bool:
    """Can rank's weights be random-initialised straight into HBM? Only when its program
    re-fills nothing in the steady state: every refill of an evicted/overwritten group must
    be a real host->HBM copy (a measured cost, and capturable in a hipGraph)."""
    return steady_fill_bytes(p.programs[rank], p.param_bytes) == 0


P2P = os.environ.get("DLS_P2P", "rccl")  # cross-GPU DAG edges: "rccl" (c10d p2p) or "device" (devp2p.py)


def p2p_group(p: Plan, rank: int, device, pg, transport: Optional[str] = None):
    """The ``pg`` to hand :func:`make_executor` for a process-per-GPU job: the process group
    itself (RCCL p2p, the default), or — ``transport="device"`` / ``DLS_P2P=device`` — the
    device-initiated transport (parallel/devp2p.py: edges moved by kernels, each rank's whole
    step one hipGraph), whose arenas and mailboxes the ranks exchange as IPC handles over ``pg``
    once, when the executors are built."""
    transport = transport or P2P
    if pg is None or p.world == 1 or transport == "rccl":
        return pg
    if transport != "device":
        raise ValueError(f"unknown p2p transport {transport!r}")
    from .devp2p import DeviceP2PGroup, DeviceP2PWorld

    return DeviceP2PGroup(DeviceP2PWorld(p, device, [rank]), rank, pg=pg)


def make_executor(p: Plan, rank: int, device, store: Optional[ParamStore] = None, pg=None, use_graph: bool = True,
                  trace: bool = False, debug: bool = False, autotune: bool = True):
    """``debug=True``: validate every rank's program first (parallel/validate.py) and run the
    executor with arena canaries and output finiteness checks. ``autotune=False``: GEMM shapes
    missing from the tuning table run the kernel's heuristic config instead of being tuned first."""
    from .executor import DAGExecutor

    if debug:
        from .validate import check_plan

        dev = torch_device_type(device) == "cuda"
        transport = getattr(pg, "world", None) is not None and type(pg).__name__ in ("DeviceP2PGroup", "HostP2PGroup")
        errs = check_plan(p, device=transport, gpu=dev)
        if errs:
            raise RuntimeError("invalid plan:\n  " + "\n  ".join(errs[:20]))
    # per-model GEMM choices by the canonical preset name (aliases such as "mixtral" resolve to it)
    return DAGExecutor(p.tasks, p.programs[rank], store or make_store(p), device, model_cfg=p.cfg,
                       use_graph=use_graph, pg=pg, trace=trace, debug=debug, model_name=p.cfg.name, autotune=autotune,
                       input_parts=p.input_parts, requests=p.requests)
