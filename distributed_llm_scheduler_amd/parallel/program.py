"""Lower a placed DAG into per-GPU programs.

Input: the task list, a placement (task -> rank) and a global order (the order in which
the scheduler committed tasks — topological by construction). Output: one
:class:`Program` per rank, built identically on every rank, containing

* ``load(p)`` / ``evict(p)`` — parameter-cache traffic replayed from the scheduler's
  action trace (``scheduler.events``) or, without a trace, load-on-first-use,
* ``recv(t, src)`` / ``send(t, dst)`` — one point-to-point transfer per (cross-GPU edge
  producer, consumer rank) pair, emitted at the PRODUCER's global position on both
  ends, so every pair of ranks posts its send/recv sequence in the same order (no
  deadlock, no tag matching; RCCL p2p over one xGMI link),
* ``run(group)`` — one kernel group. Co-located producer->consumer pairs whose
  intermediate has no other consumer are fused into one group, e.g.
  ``linear+gelu`` (GEMM epilogue), ``linear+residual`` and ``attention+residual``
  (output-projection epilogue) — the fused intermediates never exist in HBM.

Memory is planned statically: every activation gets an offset in the rank's activation
arena (native best-fit arena, lifetimes from the program), every parameter group an
offset in its parameter arena (capacity = the per-GPU memory cap). Nothing is allocated
at run time, so a rank's whole program is hipGraph-capturable.
"""
from __future__ import annotations

import math
import os
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..core import native as _native
from ..core.task import Task

ALIGN = 256
AHEAD_MAX_EXTRA = 1.10  # issuing streamed loads ahead may cost at most 10 % more refill bytes
AHEAD_MAX_FILL_RATIO = 8.0  # ... and pays while refill time <= 8 x kernel time (_overlap_pays)
HOST_LINK_BPS = 56e9  # host -> HBM refill rate, one MI355X (benchmarks/bench_h2d.py)
# host (Python) work per kernel group of an eager step: Llama-3-8B 6.9 ms / 67 groups
# (benchmarks/bench_host_overhead.py with DLS_HOST_PROFILE=1)
EAGER_HOST_S_PER_GROUP = 1e-4


@dataclass
class Instr:
    op: str  # load | evict | recv | send | psend | run
    task: Optional[str] = None      # producing task (recv/send) or output task (run)
    group: Tuple[str, ...] = ()     # run: fused task ids, execution order
    kind: str = ""                  # run: fused kind (e.g. "linear+gelu")
    # recv: source rank, send: destination rank; load: >= 0 = fetch the group from this
    # rank's arena over xGMI (RCCL p2p) instead of the host image; psend: destination rank
    peer: int = -1
    param: Optional[str] = None     # load/evict/psend
    gpos: int = -1                  # position in the global task order this instruction belongs to
    param_off: int = -1             # psend: the group's offset in this rank's parameter arena
    # run/recv: indices of earlier ``send`` instructions whose buffer this instruction's
    # output region overlaps — they must complete before it writes (see _plan_send_waits)
    wait_sends: Tuple[int, ...] = ()
    # send/recv of an expert-parallel capacity edge (plan_ep_capacity): the message is the first
    # ``rows`` rows of the tensor (routed token rows packed by the sender, or an expert's compact
    # output rows) instead of the whole buffer; 0 = the whole buffer
    rows: int = 0
    # a routed hidden state's capacity edge: the experts on the expert GPU its rows are routed to,
    # and the capacity of those experts' compact outputs coming back (their return edges)
    experts: Tuple[int, ...] = ()
    erows: int = 0


@dataclass
class Program:
    rank: int
    instrs: List[Instr] = field(default_factory=list)
    act_offset: Dict[str, int] = field(default_factory=dict)   # output task -> byte offset
    act_bytes: Dict[str, int] = field(default_factory=dict)
    act_arena_bytes: int = 0
    param_offset: Dict[Tuple[int, str], int] = field(default_factory=dict)  # (load index, pid) -> offset
    param_arena_bytes: int = 0
    param_peak_bytes: int = 0
    failed_loads: List[str] = field(default_factory=list)
    n_kernels: int = 0
    # parameter groups resident (at these arena offsets) when the program starts; the
    # executor fills them once before the first step, and a warm-started program ends by
    # restoring them (epilogue loads), so it can repeat step after step
    start_resident: Dict[str, int] = field(default_factory=dict)
    end_resident: Dict[str, int] = field(default_factory=dict)      # before the epilogue
    # how the parameter residency was lowered: "cold" / "warm" (the policy's trace from an
    # empty / a warm arena) or "planned" (plan_keep_sets: kept groups + streamed groups)
    residency: str = "cold"
    prefetch: bool = False  # planned with lookahead: loads are issued ahead for a copy stream
    # co-run spans (plan_coruns): output tasks of runs the executor may issue TOGETHER at the
    # span's first run — the expert nodes of one MoE layer placed on this rank, over every
    # request — with the activation plan keeping their inputs and outputs live across the span
    coruns: List[Tuple[str, ...]] = field(default_factory=list)

    @property
    def has_comm(self) -> bool:
        return any(i.op in ("send", "recv", "psend") or (i.op == "load" and i.peer >= 0) for i in self.instrs)

    def counts(self) -> Dict[str, int]:
        c: Dict[str, int] = defaultdict(int)
        for i in self.instrs:
            c[i.op] += 1
        return dict(c)


def _fuse_kind(prev_kind: str, nxt: Task) -> Optional[str]:
    """Kind of the group formed by appending ``nxt`` to a group of kind ``prev_kind``."""
    if nxt.op is None:
        return None
    kb = nxt.op.kind
    if prev_kind in ("layernorm", "rmsnorm") and kb in ("linear", "lm_head", "attention", "qkv_proj", "swiglu_mlp") \
            and not nxt.op.attrs.get("act"):
        return f"{prev_kind}+{kb}"  # norm folded into the GEMM (in-kernel row stats + derived weights)
    base = prev_kind.split("+", 1)[1] if prev_kind.startswith(("layernorm+", "rmsnorm+")) else prev_kind
    if base == "linear" and kb == "gelu":
        return prev_kind + "+gelu"  # GELU in the GEMM epilogue
    if base in ("linear", "linear+gelu", "attention", "attn_sp", "swiglu_mlp") and kb == "residual":
        return prev_kind + "+residual"  # residual add in the (output-projection) GEMM epilogue
    return None


def _fusion(tmap: Dict[str, Task], placement: Dict[str, int], order: Sequence[str],
            consumers: Dict[str, List[str]], pos: Dict[str, int], fuse: bool):
    """Fusion: chains on one rank, consumer is the producer's only consumer, every other
    input of the consumer is produced before the producer runs. Returns (producer ->
    consumer that absorbs it, chain end / chain start -> chain)."""
    fused_into: Dict[str, str] = {}
    group_of: Dict[str, List[str]] = {}
    if not fuse:
        return fused_into, group_of
    for tid in order:
        if tid in fused_into:
            continue
        chain = [tid]
        kind = tmap[tid].op.kind if tmap[tid].op else ""
        while True:
            cons = consumers.get(chain[-1], [])
            if len(cons) != 1 or placement[cons[0]] != placement[chain[-1]]:
                break
            nxt = cons[0]
            fk = _fuse_kind(kind, tmap[nxt])
            if fk is None:
                break
            # every other input of nxt must exist before the group starts
            others = [d for d in tmap[nxt].dependencies if d != chain[-1]]
            if any(o not in placement or pos.get(o, 1 << 60) > pos[chain[0]] for o in others):
                break
            chain.append(nxt)
            kind = fk
        if len(chain) > 1:
            for a in chain[:-1]:
                fused_into[a] = chain[-1]
            group_of[chain[-1]] = chain
            group_of[chain[0]] = chain
    return fused_into, group_of


def _consumers(tmap, placement, order):
    consumers: Dict[str, List[str]] = defaultdict(list)
    for tid in order:
        for d in tmap[tid].dependencies:
            if d in placement:
                consumers[d].append(tid)
    return consumers


def build_programs(tasks: Sequence[Task], placement: Dict[str, int], order: Sequence[str], world: int,
                   param_bytes: Dict[str, int], param_cap_bytes: Optional[Dict[int, int]] = None,
                   events: Optional[Sequence[tuple]] = None, node_rank: Optional[Dict[str, int]] = None,
                   fuse: bool = True, start_resident: Optional[Dict[int, Dict[str, int]]] = None,
                   keep: Optional[Dict[int, Sequence[str]]] = None,
                   load_at: Optional[Dict[int, Dict[str, str]]] = None) -> List[Program]:
    """Build every rank's program. ``placement`` maps task id -> rank; tasks absent from it
    (failed or orphaned by the scheduler) are skipped together with their dependents.

    ``start_resident`` (rank -> {group: arena offset}): a WARM start — those groups are
    resident where they are when the program begins (the policy's loads of them become
    no-ops), and the program ends with the loads that restore exactly that state, so one
    program is the repeating steady-state step (see :func:`build_steady_programs`).

    ``keep`` (rank -> groups): PLANNED residency instead of the policy's trace on those ranks
    — the kept groups are packed at the bottom of the arena and stay resident step after
    step; every other group is streamed: loaded before its first use in the step and evicted
    after its last (see :func:`plan_keep_sets`). ``load_at`` (rank -> {streamed group: task}):
    its load is issued before that earlier task instead, so a copy stream can fill it while
    the kernels in between run (``Program.prefetch``)."""
    core = _native.load()
    if core is None:
        raise RuntimeError("native core (_dlsched_core) is required for memory planning")
    tmap = {t.id: t for t in tasks}
    pos = {tid: i for i, tid in enumerate(order)}
    order = [t for t in order if t in placement]
    consumers = _consumers(tmap, placement, order)
    fused_into, group_of = _fusion(tmap, placement, order, consumers, pos, fuse)

    # --- parameter plan per node from the scheduler trace (load-on-first-use otherwise)
    load_before: Dict[str, List[Tuple[str, str]]] = defaultdict(list)  # task -> [(op, pid)] on its rank
    if events is not None:
        pending: Dict[int, List[Tuple[str, str]]] = defaultdict(list)
        for _, act, node, item in events:
            if act in ("LOAD", "EVICT"):
                r = node_rank[node] if node_rank else int(node)
                pending[r].append((act.lower(), item))
            elif act == "RUN" and item in placement:
                r = placement[item]
                load_before[item].extend(pending.pop(r, []))

    programs: List[Program] = []
    caps = param_cap_bytes or {}
    for rank in range(world):
        prog = Program(rank)
        ins = prog.instrs
        par = core.Arena(caps.get(rank, 1 << 50), ALIGN)
        where: Dict[str, int] = {}       # resident pid -> arena offset
        last_use: Dict[str, int] = {}    # pid -> instruction index of last use (LRU)
        extent = 0

        def evict(pid):
            ins.append(Instr("evict", param=pid))
            par.release(where.pop(pid))

        kept = None if keep is None or keep.get(rank) is None else list(keep[rank])
        kept_set = set(kept or ())
        uses_left: Dict[str, int] = defaultdict(int)  # planned mode: uses of each group still ahead
        if kept is not None:
            start = {}
            for pid in kept:
                off = par.alloc(int(param_bytes.get(pid, 0)) or 1)
                if off < 0:
                    raise RuntimeError(f"rank {rank}: kept groups exceed the parameter arena at {pid}")
                start[pid] = off
                where[pid] = off
                extent = max(extent, off + (int(param_bytes.get(pid, 0)) or 1))
            for tid in order:
                if placement[tid] == rank:
                    for pid in tmap[tid].params_needed:
                        uses_left[pid] += 1
            ahead: Dict[str, List[str]] = defaultdict(list)
            for pid, tid in sorted(((load_at or {}).get(rank) or {}).items()):
                if pid not in kept_set:
                    ahead[tid].append(pid)
            prog.prefetch = bool(ahead)
        else:
            start = dict((start_resident or {}).get(rank, {}))
            for pid, off in sorted(start.items(), key=lambda kv: kv[1]):
                nbytes = int(param_bytes.get(pid, 0)) or 1
                if not par.reserve(off, nbytes):
                    raise RuntimeError(f"rank {rank}: warm-start group {pid} does not fit at offset {off}")
                where[pid] = off
                extent = max(extent, off + nbytes)
        prog.start_resident = dict(start)
        prog.residency = "planned" if kept is not None else ("warm" if start_resident is not None else "cold")

        # parameters of fused-away members whose group has not run yet: the group reads them
        # at its tail's position, so an eviction the policy decided in between is deferred
        # until the group has run (cancelled if the policy loads the group again first)
        pinned: Dict[str, int] = defaultdict(int)
        deferred: List[str] = []
        early: set = set()  # planned mode: streamed groups loaded ahead, not used yet

        def load(pid, needed):
            nonlocal extent
            nbytes = int(param_bytes.get(pid, 0)) or 1
            off = par.alloc(nbytes)
            while off < 0:
                # fragmentation (the scheduler accounts bytes, not contiguity): evict the
                # least recently used resident group this task does not need (streamed groups
                # before kept ones in planned mode), retry
                victims = sorted((q for q in where if q not in needed and not pinned.get(q)),
                                 key=lambda q: (q in kept_set, last_use.get(q, -1)))
                if not victims:
                    prog.failed_loads.append(pid)
                    return
                evict(victims[0])
                off = par.alloc(nbytes)
            where[pid] = off
            ins.append(Instr("load", param=pid))
            prog.param_offset[(len(ins) - 1, pid)] = off
            extent = max(extent, off + nbytes)

        received = set()
        emitted_group = set()
        n0 = len(ins)
        for gi, tid in enumerate(order):
            for x in ins[n0:]:
                x.gpos = gi - 1
            n0 = len(ins)
            r = placement[tid]
            t = tmap[tid]
            if r == rank:
                needed = set(t.params_needed)
                if events is not None and kept is None:  # replay the policy's cache decisions
                    for op, pid in load_before.get(tid, []):
                        if op == "evict" and pid in where and pid not in needed:
                            if pinned.get(pid):
                                if pid not in deferred:
                                    deferred.append(pid)
                            else:
                                evict(pid)
                        elif op == "load":
                            if pid in deferred:
                                deferred.remove(pid)  # still resident: the reload is free
                            elif pid not in where:
                                load(pid, needed | {q for q, c in pinned.items() if c})
                for pid in sorted(needed):
                    if pid not in where:
                        load(pid, needed | early | {q for q, c in pinned.items() if c})
                    last_use[pid] = len(ins)
                if kept is not None:  # streamed groups issued ahead, after this task's own loads
                    early -= needed
                    for pid in ahead.get(tid, ()):
                        if pid not in where:
                            load(pid, needed | early | {q for q, c in pinned.items() if c})
                            early.add(pid)
                if kept is not None:  # streamed group after its last use: out once its group has run
                    for pid in sorted(needed):
                        uses_left[pid] -= 1
                        if uses_left[pid] == 0 and pid not in kept_set and pid not in deferred:
                            deferred.append(pid)
                if tid in fused_into:
                    for pid in needed:
                        pinned[pid] += 1
                    continue  # executed as part of its consumer's group
                grp = tuple(group_of.get(tid, [tid]))
                if grp in emitted_group:
                    continue
                emitted_group.add(grp)
                kind = _group_kind(tmap, grp)
                ins.append(Instr("run", task=grp[-1], group=grp, kind=kind))
                prog.n_kernels += 1
                for member in grp[:-1]:
                    for pid in tmap[member].params_needed:
                        pinned[pid] -= 1
                for pid in [q for q in deferred if not pinned.get(q)]:
                    deferred.remove(pid)
                    if pid in where:
                        evict(pid)
                dsts = sorted({placement[c] for c in consumers.get(grp[-1], []) if placement[c] != rank})
                for dst in dsts:
                    ins.append(Instr("send", task=grp[-1], peer=dst))
            else:
                if tid in fused_into:
                    continue
                if any(placement[c] == rank for c in consumers.get(tid, [])) and tid not in received:
                    ins.append(Instr("recv", task=tid, peer=r))
                    received.add(tid)
        for x in ins[n0:]:
            x.gpos = len(order) - 1
        n0 = len(ins)
        prog.end_resident = dict(where)
        if start_resident is not None or kept is not None:  # epilogue: restore the start state
            for pid in [q for q in where if start.get(q) != where[q]]:
                evict(pid)
            for pid, off in sorted(start.items(), key=lambda kv: kv[1]):
                if pid in where:
                    continue
                if not par.reserve(off, int(param_bytes.get(pid, 0)) or 1):
                    raise RuntimeError(f"rank {rank}: cannot restore {pid} at offset {off}")
                where[pid] = off
                ins.append(Instr("load", param=pid))
                prog.param_offset[(len(ins) - 1, pid)] = off
        for x in ins[n0:]:
            x.gpos = len(order)
        if EP_CAPACITY > 0:
            plan_ep_capacity(prog, rank, tmap, placement, consumers, EP_CAPACITY)
        prog.param_peak_bytes = par.peak
        prog.param_arena_bytes = extent
        sinks = {t for t in order if not consumers.get(t)}
        prog.coruns = plan_coruns(prog, tmap)
        _plan_activations(core, prog, tmap, sinks)
        _plan_send_waits(prog)
        if prog.failed_loads:
            raise RuntimeError(
                f"rank {rank}: parameter groups {sorted(set(prog.failed_loads))} do not fit the fragmented "
                f"parameter arena ({caps.get(rank, 0)} B cap) even after evicting every group their task "
                "does not need; raise the cap or use a policy that places fewer parameters on this rank")
        programs.append(prog)
    return programs


# Expert-parallel edges on the default (RCCL) transport: a hidden state sent to an expert GPU
# carries the token rows routed to that GPU's experts, packed by the sender into a buffer of
# ceil(EP_CAPACITY * M * k * n / E) rows (n experts there), and an expert's compact output goes back
# in an edge of ceil(EP_CAPACITY * M * k / E) rows — fixed-size messages (an RCCL receive must know
# its size when it is posted; the routing lives on the device), ~EP_CAPACITY x the routed bytes
# instead of M rows each. A layer whose routing overflows a capacity is detected on the device
# (DAGExecutor.ep_overflow) and that edge widened to the whole buffer. DLS_EP_CAPACITY=0: whole
# buffers always (the round-5 edges).
EP_CAPACITY = float(os.environ.get("DLS_EP_CAPACITY", "1.25"))
EP_ROWS_ALIGN = 8


def ep_capacity_rows(M: int, k: int, n_exp: int, E: int, factor: float) -> int:
    """Rows of a capacity edge to n_exp of E experts: factor x the expected routed rows M*k*n/E,
    at most every row a routing can send there (a token counts once per expert it picks)."""
    rows = math.ceil(factor * M * k * n_exp / E / EP_ROWS_ALIGN) * EP_ROWS_ALIGN
    return max(EP_ROWS_ALIGN, min(M * min(k, n_exp), rows))


def ep_routed_in(h: str, dst: int, tmap: Dict[str, Task], placement: Dict[str, int],
                 consumers: Dict[str, List[str]]) -> Optional[List[Task]]:
    """The expert nodes on ``dst`` that read ``h`` as their tokens, if they are h's only consumers
    there (the edge h -> dst then carries routed rows only), else None."""
    us = [tmap[c] for c in consumers.get(h, []) if placement.get(c) == dst]
    if us and all(u.op is not None and u.op.kind == "moe_expert" and u.op.inputs[0] == h for u in us):
        return us
    return None


def ep_routed_out(x: str, dst: int, tmap: Dict[str, Task], placement: Dict[str, int],
                  consumers: Dict[str, List[str]]) -> bool:
    """An expert's output whose consumers on ``dst`` are all MoE combines (compact rows)."""
    t = tmap[x]
    us = [tmap[c] for c in consumers.get(x, []) if placement.get(c) == dst]
    return bool(us) and t.op is not None and t.op.kind == "moe_expert" and all(
        u.op is not None and u.op.kind == "moe_combine" for u in us)


def _ep_hidden_rows(h: str, src: int, dst: int, tmap, placement, consumers, factor: float):
    """(rows, experts, router) of the capacity edge h: src -> dst, or None when that edge stays a
    whole buffer: its consumers there are not all experts reading h as tokens, their routing is
    not computed on src, or the capacity would not be smaller than the buffer (several experts
    on one GPU count a token once per expert it picks)."""
    us = ep_routed_in(h, dst, tmap, placement, consumers)
    t = tmap[h]
    if not us or t.op is None or not t.op.out_shape:
        return None
    r = us[0].op.inputs[1]
    if placement.get(r) != src or any(u.op.inputs[1] != r for u in us):
        return None
    M = math.prod(t.op.out_shape[:-1])
    a = us[0].op.attrs
    experts = tuple(sorted({u.op.attrs["expert"] for u in us}))
    rows = ep_capacity_rows(M, a["top_k"], len(experts), a["n_experts"], factor)
    if rows >= M:
        return None
    return rows, experts, r, ep_capacity_rows(M, a["top_k"], 1, a["n_experts"], factor)


def plan_ep_capacity(prog: Program, rank: int, tmap: Dict[str, Task], placement: Dict[str, int],
                     consumers: Dict[str, List[str]], factor: float) -> int:
    """Turn this rank's expert-parallel edges into capacity edges (``Instr.rows``) and move each
    routed hidden state's send / receive right after the router logits' send / receive between
    the same two ranks — the sender packs the rows once its routing exists, and both ends post
    in the same order (RCCL pairs a rank pair's messages by posting order). An expert's output
    going back is a capacity edge exactly when its tokens came through one. Returns the number
    of capacity edges. Parameter-load indices (``param_offset``) follow the moves."""
    ins = prog.instrs
    moves: Dict[int, Tuple[str, str]] = {}  # instruction -> (op, router task) it is posted after
    n = 0
    for i, x in enumerate(ins):
        if x.op not in ("send", "recv"):
            continue
        src, dst = (rank, x.peer) if x.op == "send" else (x.peer, rank)
        hid = _ep_hidden_rows(x.task, src, dst, tmap, placement, consumers, factor)
        if hid is not None:
            x.rows, x.experts, r, x.erows = hid
            moves[i] = (x.op, r)
            n += 1
            continue
        t = tmap[x.task]
        if ep_routed_out(x.task, dst, tmap, placement, consumers):
            h = t.op.inputs[0]
            if placement.get(h) != dst:
                continue
            back = _ep_hidden_rows(h, dst, src, tmap, placement, consumers, factor)  # its tokens' edge
            if back is not None and t.op.attrs["expert"] in back[1]:
                x.rows = back[3]
                n += 1
    if not moves:
        return n
    order = [i for i in range(len(ins)) if i not in moves]
    for i, (op, r) in sorted(moves.items()):
        peer = ins[i].peer
        anchor = next((k for k, j in enumerate(order) if ins[j].op == op and ins[j].task == r and ins[j].peer == peer),
                      None)
        if anchor is None:
            raise RuntimeError(f"rank {rank}: routed edge {ins[i].task} has no {op} of its router {r} to follow")
        # after the router's message and any routed states already placed behind it
        k = anchor + 1
        while k < len(order) and order[k] in moves and moves[order[k]] == (op, r) and ins[order[k]].peer == peer:
            k += 1
        order.insert(k, i)
        ins[i].gpos = ins[order[anchor]].gpos
    new_index = {old: new for new, old in enumerate(order)}
    prog.instrs = [ins[j] for j in order]
    prog.param_offset = {(new_index[i], pid): off for (i, pid), off in prog.param_offset.items()}
    return n


def moe_batched_ids(prog: Program, tmap: Dict[str, Task]) -> set:
    """Expert nodes that run as ONE grouped launch pair per MoE layer (DAGExecutor._plan_moe_batches
    on the GPU): every expert of a layer back to back on this rank (only parameter loads between
    them), in a program without evictions or peer parameter loads."""
    ins = prog.instrs
    out: set = set()
    if any(i.op == "evict" or (i.op == "load" and i.peer >= 0) for i in ins):
        return out

    def expert_of(j):
        x = ins[j]
        if x.op != "run" or len(x.group) != 1:
            return None
        t = tmap[x.group[0]]
        return t if t.op is not None and t.op.kind == "moe_expert" else None

    i = 0
    while i < len(ins):
        t0 = expert_of(i)
        if t0 is None:
            i += 1
            continue
        key = tuple(t0.op.inputs[:2])
        members, j = [i], i + 1
        while j < len(ins):
            t = expert_of(j)
            if ins[j].op == "load":
                pass
            elif t is not None and tuple(t.op.inputs[:2]) == key:
                members.append(j)
            else:
                break
            j += 1
        experts = sorted(tmap[ins[m].group[0]].op.attrs["expert"] for m in members)
        if len(members) > 1 and experts == list(range(t0.op.attrs["n_experts"])):
            out |= {ins[m].group[0] for m in members}
        i = j
    return out


def device_routed_edges(prog: Program, tmap: Dict[str, Task], batched: set = frozenset()):
    """The device transport's routed receives on this rank (DAGExecutor._plan_routed_edges and
    validate.device_deadlock_check share this rule): {hidden state: its local expert nodes} for a
    received hidden state whose every local consumer is an expert reading it as its tokens and
    not part of a whole-layer batch (``batched``), and the received expert outputs whose every
    local consumer is a MoE combine."""
    users: Dict[str, List[Task]] = defaultdict(list)
    for ins in prog.instrs:
        if ins.op == "run":
            for tid in ins.group:
                for d in tmap[tid].dependencies:
                    users[d].append(tmap[tid])
    routed_in: Dict[str, List[Task]] = {}
    routed_out: set = set()
    for x in {i.task for i in prog.instrs if i.op == "recv"}:
        us = users.get(x, [])
        if us and all(u.op is not None and u.op.kind == "moe_expert" and u.op.inputs[0] == x
                      and u.id not in batched for u in us):
            routed_in[x] = us
        elif us and all(u.op is not None and u.op.kind == "moe_combine" for u in us) \
                and tmap[x].op is not None and tmap[x].op.kind == "moe_expert":
            routed_out.add(x)
    return routed_in, routed_out


def _group_kind(tmap: Dict[str, Task], grp: Tuple[str, ...]) -> str:
    kind = tmap[grp[0]].op.kind if tmap[grp[0]].op else "noop"
    for nxt in grp[1:]:
        kind = _fuse_kind(kind, tmap[nxt]) or kind
    return kind


def _moe_layer_key(tmap: Dict[str, Task], ins: Instr) -> Optional[str]:
    """The MoE layer an expert run belongs to (its router's id without the request prefix)."""
    if ins.op != "run" or len(ins.group) != 1:
        return None
    op = tmap[ins.group[0]].op
    if op is None or op.kind != "moe_expert":
        return None
    r = op.inputs[1]
    head, _, rest = r.partition("/")
    return rest if rest and head[:1] == "r" and head[1:].isdigit() else r


def plan_coruns(prog: Program, tmap: Dict[str, Task]) -> List[Tuple[str, ...]]:
    """Spans of expert runs that can be issued as ONE grouped launch pair at the span's first
    run: consecutive runs of one MoE layer's expert nodes (any expert, any request — with
    data-parallel attention every request's tokens reach the same expert GPU in the same
    layer), with only sends, parameter loads and receives no member reads between them, and
    every member's inputs present before the first member. Then each expert's weights stream
    once per layer for all requests instead of once per request. Not planned for programs
    that evict or fetch parameters from peers (regions must not move inside a span)."""
    ins = prog.instrs
    if any(x.op == "evict" or x.op == "psend" or (x.op == "load" and x.peer >= 0) for x in ins):
        return []
    defined: Dict[str, int] = {}
    spans: List[Tuple[str, ...]] = []
    i = 0
    while i < len(ins):
        key = _moe_layer_key(tmap, ins[i])
        if key is None:
            if ins[i].op in ("run", "recv"):
                defined.setdefault(ins[i].task, i)
            i += 1
            continue
        a, members, j = i, [i], i + 1
        defined.setdefault(ins[i].task, i)
        while j < len(ins):
            x = ins[j]
            if x.op in ("send", "load"):
                j += 1
                continue
            if x.op == "recv":
                defined.setdefault(x.task, j)
                j += 1
                continue
            if _moe_layer_key(tmap, x) != key or any(defined.get(d, a) >= a for d in tmap[x.group[0]].dependencies):
                break
            members.append(j)
            defined.setdefault(x.task, j)
            j += 1
        if len(members) > 1:
            spans.append(tuple(ins[m].task for m in members))
        i = members[-1] + 1
    return spans


def _plan_activations(core, prog: Program, tmap: Dict[str, Task], sinks=frozenset()) -> None:
    """Static activation lifetimes -> offsets in the rank's activation slab. DAG outputs
    (``sinks``: tasks nobody consumes, e.g. the logits of every request) stay live. A co-run
    span (``prog.coruns``) allocates every member's output at its first member and keeps every
    member's inputs live to its last member."""
    # last use index of each activation on this rank
    last_use: Dict[str, int] = {}
    run_at = {ins.task: i for i, ins in enumerate(prog.instrs) if ins.op == "run"}
    alloc_at: Dict[int, List[str]] = {}
    early: set = set()
    span_end: Dict[str, int] = {}
    for span in prog.coruns:
        idx = [run_at[t] for t in span]
        alloc_at[idx[0]] = list(span)
        early |= set(span[1:])
        for t in span:
            span_end[t] = idx[-1]
    for i, ins in enumerate(prog.instrs):
        if ins.op == "run":
            for tid in ins.group:
                for d in tmap[tid].dependencies:
                    last_use[d] = max(last_use.get(d, i), span_end.get(ins.task, i))
            last_use.setdefault(ins.task, i)
        elif ins.op in ("send", "recv"):
            last_use[ins.task] = max(last_use.get(ins.task, i), i)
    act = core.Arena(1 << 50, ALIGN)
    frees: Dict[int, List[str]] = defaultdict(list)
    for tid, i in last_use.items():
        if tid not in sinks:
            frees[i].append(tid)
    live: Dict[str, int] = {}
    extent = 0
    for i, ins in enumerate(prog.instrs):
        if ins.op in ("run", "recv") and ins.task not in early:
            for tid in alloc_at.get(i, [ins.task]):
                nbytes = max(int(tmap[tid].out_bytes), 1)
                off = act.alloc(nbytes)
                prog.act_offset[tid] = off
                prog.act_bytes[tid] = nbytes
                live[tid] = off
                extent = max(extent, off + nbytes)
        for tid in frees.get(i, []):
            if tid in live:
                act.release(live.pop(tid))
    prog.act_arena_bytes = extent  # slab size = highest byte any activation reaches


def _plan_send_waits(prog: Program) -> None:
    """A ``send`` reads its buffer asynchronously (RCCL stream of that peer pair) until the
    receiver has taken it; the activation plan frees the buffer at the send, so a later
    ``run`` OR ``recv`` (another peer pair, another RCCL stream) may be given the same
    bytes. Every such writer gets the overlapping in-flight sends in ``wait_sends``; the
    executor completes them before the write, and the validator checks the list and the
    deadlock freedom of the waits (parallel/validate.py)."""
    inflight: List[Tuple[int, int, int]] = []  # (send index, lo, hi)
    run_at = {ins.task: i for i, ins in enumerate(prog.instrs) if ins.op == "run"}
    together: Dict[int, List[int]] = {}  # a co-run span's members write at its first run
    later: set = set()
    for span in prog.coruns:
        idx = [run_at[t] for t in span]
        together[idx[0]] = idx
        later |= set(idx[1:])
    for i, ins in enumerate(prog.instrs):
        if ins.op == "send":
            lo = prog.act_offset[ins.task]
            inflight.append((i, lo, lo + prog.act_bytes[ins.task]))
            continue
        if i in later:
            continue
        for k in together.get(i, [i]):
            w = prog.instrs[k]
            if w.op in ("run", "recv") and inflight and w.task in prog.act_offset:
                lo = prog.act_offset[w.task]
                hi = lo + prog.act_bytes[w.task]
                hit = [s for s in inflight if s[1] < hi and lo < s[2]]
                if hit:
                    w.wait_sends = tuple(s[0] for s in hit)
                    inflight = [s for s in inflight if s not in hit]


def plan_keep_sets(tasks: Sequence[Task], placement: Dict[str, int], order: Sequence[str], world: int,
                   param_bytes: Dict[str, int], budget: Dict[int, float], param_units: Dict[str, float],
                   param_cap_bytes: Optional[Dict[int, int]] = None, fuse: bool = True,
                   lookahead: int = 0) -> Tuple[Dict[int, List[str]], Dict[int, Dict[str, str]]]:
    """Steady-state residency for a repeating step: per rank, the parameter groups to keep
    resident; the rest are streamed (loaded before first use, evicted after last use).

    Every group is used once per step, so a kept group saves its whole refill and the
    per-step refill is the streamed bytes. The constraint is that the kept groups plus the
    streamed groups live at the same moment fit the budget (``budget[rank]``, the policy's
    cost units, e.g. the node cap minus the largest activation requirement; and the byte
    arena ``param_cap_bytes``). Recency-based eviction (the policy's one-pass trace) streams
    whatever came last — for Llama-3-8B the 1.05 GB LM head, whose buffer then displaces ~1 GB
    of layers. Here groups are kept greedily by refill bytes per budget unit, largest first,
    so the streaming buffer is sized by the SMALL groups that remain.

    ``lookahead`` = k > 0: a streamed group's load is issued at the first use of the streamed
    group k places before it (second return value: rank -> {group: task}, for
    :func:`build_programs`' ``load_at``), and the keep set is chosen with those longer
    lifetimes. Returns (rank -> kept groups, rank -> load positions).
    """
    import bisect

    import numpy as np

    tmap = {t.id: t for t in tasks}
    pos = {tid: i for i, tid in enumerate(order)}
    order = [t for t in order if t in placement]
    consumers = _consumers(tmap, placement, order)
    fused_into, _ = _fusion(tmap, placement, order, consumers, pos, fuse)
    at = {tid: i for i, tid in enumerate(order)}

    def tail(tid):
        while tid in fused_into:
            tid = fused_into[tid]
        return tid

    caps = param_cap_bytes or {}
    out: Dict[int, List[str]] = {}
    where_load: Dict[int, Dict[str, str]] = {}
    for rank in range(world):
        span: Dict[str, List[int]] = {}
        for tid in order:
            if placement[tid] != rank:
                continue
            lo, hi = at[tid], at[tail(tid)]
            for pid in tmap[tid].params_needed:
                sp = span.setdefault(pid, [lo, hi])
                sp[0], sp[1] = min(sp[0], lo), max(sp[1], hi)
        n = max(len(order), 1)
        units = {pid: float(param_units.get(pid, 0.0)) for pid in span}
        nbytes = {pid: float(_aligned(param_bytes.get(pid, 0))) for pid in span}
        cap_u, cap_b = float(budget.get(rank, 0.0)), float(caps.get(rank, 1 << 50))
        ratio = {q: float(param_bytes.get(q, 0)) / max(units[q], 1e-30) for q in span}
        top = max(ratio.values(), default=1.0) or 1.0
        # replicas (ranks with the same groups) keep different equal groups: each one's streamed
        # groups are then resident on a peer, and plan_peer_fills fetches them over xGMI
        prio = _spread(sorted(span, key=lambda q: (-round(ratio[q] / top, 6), -nbytes[q], span[q][0], q)),
                       key=lambda q: (round(ratio[q] / top, 6), nbytes[q]), shift=rank)

        def choose(spans):
            live_u, live_b = np.zeros(n), np.zeros(n)
            for pid, (lo, hi) in spans.items():
                live_u[lo:hi + 1] += units[pid]
                live_b[lo:hi + 1] += nbytes[pid]
            keep_u = keep_b = 0.0
            kept: List[str] = []
            for pid in prio:
                lo, hi = spans[pid]
                tu, tb = live_u.copy(), live_b.copy()
                tu[lo:hi + 1] -= units[pid]
                tb[lo:hi + 1] -= nbytes[pid]
                if keep_u + units[pid] + max(tu.max(), 0.0) <= cap_u + 1e-9 and \
                        keep_b + nbytes[pid] + max(tb.max(), 0.0) <= cap_b:
                    kept.append(pid)
                    keep_u += units[pid]
                    keep_b += nbytes[pid]
                    live_u, live_b = tu, tb
            return kept

        kept = choose(span)
        if lookahead > 0:
            # a streamed group is live from the first use of the streamed group `lookahead`
            # places before it (its load is issued there); the streamed sequence is taken from
            # the plain choice, then the keep set is re-chosen with the longer lifetimes
            kset = set(kept)
            firsts = sorted(span[q][0] for q in span if q not in kset)
            ext = {}
            for pid, (lo, hi) in span.items():
                k = bisect.bisect_left(firsts, lo)  # streamed groups first used before this one
                ext[pid] = [min(firsts[k - lookahead], lo) if k >= lookahead else lo, hi]
            kept = choose(ext)
            where_load[rank] = {q: order[ext[q][0]] for q in span if q not in set(kept) and ext[q][0] < span[q][0]}
        out[rank] = sorted(kept, key=lambda q: (span[q][0], q))
    return out, where_load


def _spread(items: List[str], key, shift: int = 0) -> List[str]:
    """Reorder each run of equal-``key`` items (in step order) by the bit-reversed run index,
    so any prefix of the run — the groups the greedy keeps — is spread evenly over the step,
    and so are the streamed rest: refills then alternate with kernels all through the step
    instead of bunching (e.g. the 32 equal attention out-projections of Llama-3-8B). ``shift``
    rotates the run by that many items first: the last quarter of a bit-reversed order is the
    items at 3 mod 4, so ranks 0..3 shifted by 0..3 stream disjoint quarters (a rotation by a
    power-of-two fraction of the run would leave the kept set unchanged)."""
    out: List[str] = []
    i = 0
    while i < len(items):
        j = i
        while j < len(items) and key(items[j]) == key(items[i]):
            j += 1
        run = items[i:j]
        r = shift % max(len(run), 1)
        run = run[r:] + run[:r]
        bits = max(1, (len(run) - 1).bit_length())
        rev = lambda x: int(format(x, f"0{bits}b")[::-1], 2)  # noqa: E731
        out += [run[k] for k in sorted(range(len(run)), key=rev)]
        i = j
    return out


def _aligned(nbytes) -> int:
    nbytes = int(nbytes) or 1
    return (nbytes + ALIGN - 1) // ALIGN * ALIGN


def build_steady_programs(tasks: Sequence[Task], placement: Dict[str, int], order: Sequence[str], world: int,
                          param_bytes: Dict[str, int], param_cap_bytes: Optional[Dict[int, int]] = None,
                          events: Optional[Sequence[tuple]] = None, node_rank: Optional[Dict[str, int]] = None,
                          fuse: bool = True, rounds: int = 3,
                          planned: Optional[Tuple[Dict[int, float], Dict[str, float]]] = None,
                          lookahead: int = 0, force_ahead: bool = False) -> List[Program]:
    """Programs for the repeating step. The cold lowering (empty arenas) plans every load at
    the offsets an empty arena gives; in steady state the arena instead holds whatever the
    previous step left, so many of those loads would overwrite resident groups and re-fill
    them. Instead: start each rank from the state the previous lowering ENDS in (warm start),
    restore it at the end, and iterate a few rounds; keep the programs that re-fill the fewest
    bytes per step (every load of a warm program is a real copy).

    ``planned`` = (budget per rank, budget units per group): a policy whose memory model is
    the repeating step (EFT) also offers the :func:`plan_keep_sets` residency as a candidate;
    when it wins and ``lookahead`` > 0, the programs issue its streamed loads that far ahead
    (a copy stream overlaps them with the kernels; a few more bytes stream) — where that pays
    (``_overlap_pays``), or always with ``force_ahead`` (``DLS_PREFETCH=1``)."""
    progs = build_programs(tasks, placement, order, world, param_bytes, param_cap_bytes, events, node_rank, fuse)
    # the cold lowering repeated as is (no start state) is a candidate too
    best, best_bytes = progs, sum(steady_fill_bytes(p, param_bytes) for p in progs)
    for _ in range(rounds):
        warm = build_programs(tasks, placement, order, world, param_bytes, param_cap_bytes, events, node_rank, fuse,
                              start_resident={p.rank: p.end_resident for p in progs})
        nbytes = sum(steady_fill_bytes(p, param_bytes) for p in warm)
        if nbytes < best_bytes:
            best, best_bytes = warm, nbytes
        if all(w.end_resident == p.end_resident for w, p in zip(warm, progs)):
            break  # fixed point: the next round would lower the same programs
        progs = warm
    if planned is not None and best_bytes > 0:
        cand, nbytes = _planned_programs(tasks, placement, order, world, param_bytes, param_cap_bytes, node_rank,
                                         fuse, planned, 0)
        if cand is not None and nbytes < best_bytes:
            best, best_bytes = cand, nbytes
            if lookahead > 0:  # the same residency with loads issued ahead for a copy stream
                ahead, ab = _planned_programs(tasks, placement, order, world, param_bytes, param_cap_bytes,
                                              node_rank, fuse, planned, lookahead)
                # the longer lifetimes displace kept groups: worth it while the extra refill is
                # small next to the kernel time it overlaps (Llama-3-8B: +4 % bytes)
                if ahead is not None and (force_ahead or (ab <= AHEAD_MAX_EXTRA * nbytes and
                                                          _overlap_pays(tasks, placement, ahead, param_bytes))):
                    best = ahead
    return best


def _overlap_pays(tasks, placement, progs, param_bytes) -> bool:
    """Issue streamed loads ahead only while the refill time is within AHEAD_MAX_FILL_RATIO x
    the rank's kernel time (the DAG's compute estimates): overlap can hide at most the kernel
    time, and a copy-engine fill beside kernels runs ~5 % below the in-order pull kernel.
    Measured on MI355X, Llama-3-8B (kernels ~9.7 ms) at 90 / 80 / 60 % cap: refill/kernel
    ratio 1.6 / 5.3 / 12.5 -> 23.0 -> 20.4, 54.0 -> 51.4, 115.2 -> 118.2 ms per step. The
    overlapped step runs eagerly (no hipGraph), so the kernel time must also cover the host's
    launch work (EAGER_HOST_S_PER_GROUP per kernel group), else the step turns host-bound."""
    comp: Dict[int, float] = defaultdict(float)
    for t in tasks:
        if t.id in placement:
            comp[placement[t.id]] += float(t.compute_time)
    for pr in progs:
        fill_s = steady_fill_bytes(pr, param_bytes) / HOST_LINK_BPS
        c = comp.get(pr.rank, 0.0)
        if fill_s > AHEAD_MAX_FILL_RATIO * max(c, 1e-9) or c < EAGER_HOST_S_PER_GROUP * pr.n_kernels:
            return False
    return True


def _planned_programs(tasks, placement, order, world, param_bytes, param_cap_bytes, node_rank, fuse, planned,
                      lookahead):
    """(programs, steady-state fill bytes) of the planned keep set, or (None, 0)."""
    keep, load_at = plan_keep_sets(tasks, placement, order, world, param_bytes, planned[0], planned[1],
                                   param_cap_bytes, fuse, lookahead=lookahead)
    for _ in range(8):  # best-fit fragmentation of the streaming region: shed kept groups
        try:
            progs = build_programs(tasks, placement, order, world, param_bytes, param_cap_bytes, None, node_rank,
                                   fuse, keep=keep, load_at=load_at)
        except RuntimeError:
            keep = {r: k[:-1] for r, k in keep.items()}
            continue
        return progs, sum(steady_fill_bytes(p, param_bytes) for p in progs)
    return None, 0


def steady_fill_bytes(prog: Program, param_bytes: Dict[str, int], steps: int = 2,
                      victim_reuse: Optional[bool] = None) -> int:
    """Parameter bytes the executor copies in the ``steps``-th repetition of the program:
    a ``load`` costs nothing when its arena region still holds the group from before and it
    was not evicted since (the executor's steady-state residency, DAGExecutor._fill), else
    one copy of the group.
    A warm-started program's start groups are valid from the executor's one-time fill."""
    if victim_reuse is None:
        victim_reuse = os.environ.get("DLS_VICTIM_REUSE", "0") == "1"  # executor.VICTIM_REUSE
    valid: List[Tuple[int, int, str]] = [(off, int(param_bytes.get(pid, 0)) or 1, pid)
                                         for pid, off in prog.start_resident.items()]
    filled = 0
    for _ in range(steps):
        filled = 0
        for i, ins in enumerate(prog.instrs):
            if ins.op == "evict":  # an evicted group's bytes are gone (DAGExecutor._evict)
                if not victim_reuse:
                    valid = [r for r in valid if r[2] != ins.param]
                continue
            if ins.op != "load":
                continue
            off = prog.param_offset.get((i, ins.param))
            if off is None:
                continue
            size = int(param_bytes.get(ins.param, 0)) or 1
            if (off, size, ins.param) in valid:
                continue
            valid = [r for r in valid if r[0] + r[1] <= off or off + size <= r[0]]
            valid.append((off, size, ins.param))
            filled += size
    return filled


def _fill_loads(prog: Program, param_bytes: Dict[str, int]) -> set:
    """Indices of the load instructions that copy bytes in the steady state (every step)."""
    valid = [(off, int(param_bytes.get(pid, 0)) or 1, pid) for pid, off in prog.start_resident.items()]
    fills = set()
    for step in range(2):
        for i, ins in enumerate(prog.instrs):
            if ins.op == "evict":
                valid = [r for r in valid if r[2] != ins.param]
            elif ins.op == "load":
                off = prog.param_offset.get((i, ins.param))
                if off is None:
                    continue
                size = int(param_bytes.get(ins.param, 0)) or 1
                if (off, size, ins.param) in valid:
                    continue
                valid = [r for r in valid if r[0] + r[1] <= off or off + size <= r[0]]
                valid.append((off, size, ins.param))
                if step == 1:
                    fills.add(i)
    return fills


def plan_peer_fills(programs: List[Program], tasks: Sequence[Task], param_bytes: Dict[str, int]) -> int:
    """Parameter refills over xGMI: a steady-state refill of group g on rank B at global
    position k is fetched from a rank A that holds g at k (loaded earlier in the step, not yet
    evicted) — an RCCL p2p transfer over one xGMI link (≈153 GB/s) instead of the host link
    (≈52 GB/s measured). A posts a ``psend`` at position k (ahead of its receives at k, so the
    per-pair message order matches on both ends); B's load becomes a receive into its region;
    A's later writes into that region wait for the send. Only between ranks that use g the same
    way (same fused kernel kinds): a weight is transformed in place for its fused kernel
    (folded norm, SwiGLU interleave, RoPE order), so bytes are exchanged only in equal form.
    Senders are spread over the holders (fewest sends first). Returns the number of fetches."""
    tmap = {t.id: t for t in tasks}
    if len(programs) < 2:
        return 0
    # how each rank uses each group (the in-place transform a fused kernel applies)
    sig: Dict[Tuple[int, str], frozenset] = defaultdict(frozenset)
    for pr in programs:
        acc: Dict[str, set] = defaultdict(set)
        for ins in pr.instrs:
            if ins.op == "run":
                for j, tid in enumerate(ins.group):
                    for pid in tmap[tid].params_needed:
                        acc[pid].add((ins.kind, j, tmap[tid].op.kind if tmap[tid].op else ""))
        for pid, v in acc.items():
            sig[(pr.rank, pid)] = frozenset(v)
    # residency intervals (start gpos, end gpos, offset): resident strictly inside (start, end)
    spans: Dict[str, List[Tuple[int, float, int, int]]] = defaultdict(list)  # pid -> (s, e, off, rank)
    for pr in programs:
        open_: Dict[str, Tuple[int, int]] = {pid: (-2, off) for pid, off in pr.start_resident.items()}
        for i, ins in enumerate(pr.instrs):
            if ins.op == "load":
                off = pr.param_offset.get((i, ins.param))
                if off is not None:
                    open_[ins.param] = (ins.gpos, off)
            elif ins.op == "evict" and ins.param in open_:
                s0, off = open_.pop(ins.param)
                spans[ins.param].append((s0, ins.gpos, off, pr.rank))
        for pid, (s0, off) in open_.items():
            spans[pid].append((s0, float("inf"), off, pr.rank))
    sends_by: Dict[int, int] = defaultdict(int)
    plan: Dict[int, List[Tuple[int, str, int, int]]] = defaultdict(list)  # holder -> (gpos, pid, dst, off)
    n = 0
    for pr in programs:
        for i in sorted(_fill_loads(pr, param_bytes)):
            ins = pr.instrs[i]
            k, g = ins.gpos, ins.param
            holders = [(sends_by[r], r, off) for s0, e, off, r in spans[g]
                       if r != pr.rank and s0 < k < e and sig[(r, g)] == sig[(pr.rank, g)]]
            if not holders:
                continue
            _, a, off = min(holders)
            ins.peer = a
            sends_by[a] += 1
            plan[a].append((k, g, pr.rank, off))
            n += 1
    for pr in programs:
        if plan.get(pr.rank):
            _insert_psends(pr, plan[pr.rank], param_bytes)
    return n


def _insert_psends(pr: Program, sends: List[Tuple[int, str, int, int]], param_bytes: Dict[str, int]) -> None:
    """Insert psend(g -> dst) at global position k: before the first instruction of a later
    position, and before this rank's receives at k. Instruction indices change, so the
    index-keyed parameter offsets and the send waits are rebuilt."""
    sends = sorted(sends)
    old = pr.instrs
    new: List[Instr] = []
    remap: Dict[int, int] = {}
    si = 0
    for i, ins in enumerate(old):
        while si < len(sends) and (ins.gpos > sends[si][0] or (ins.gpos == sends[si][0] and ins.op == "recv")):
            k, g, dst, off = sends[si]
            new.append(Instr("psend", param=g, peer=dst, gpos=k, param_off=off))
            si += 1
        remap[i] = len(new)
        new.append(ins)
    for k, g, dst, off in sends[si:]:
        new.append(Instr("psend", param=g, peer=dst, gpos=k, param_off=off))
    pr.instrs = new
    pr.param_offset = {(remap[i], pid): off for (i, pid), off in pr.param_offset.items()}
    pr.coruns = []  # (regions move between peers: every run issues at its own position)
    for ins in new:
        ins.wait_sends = ()
    _plan_send_waits(pr)
    _plan_psend_waits(pr, param_bytes)


def _plan_psend_waits(pr: Program, param_bytes: Dict[str, int]) -> None:
    """A psend reads its group's region until the receiver took it: a later load into an
    overlapping region (a host fill or a peer receive) waits for it first."""
    inflight: List[Tuple[int, int, int]] = []
    for i, ins in enumerate(pr.instrs):
        if ins.op == "psend":
            inflight.append((i, ins.param_off, ins.param_off + (int(param_bytes.get(ins.param, 0)) or 1)))
        elif ins.op == "load" and inflight:
            off = pr.param_offset.get((i, ins.param))
            if off is None:
                continue
            hi = off + (int(param_bytes.get(ins.param, 0)) or 1)
            hit = [x for x in inflight if x[1] < hi and off < x[2]]
            if hit:
                ins.wait_sends = tuple(ins.wait_sends) + tuple(x[0] for x in hit)
                inflight = [x for x in inflight if x not in hit]
