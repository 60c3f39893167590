"""Static checks of lowered per-GPU programs — the "debug mode that validates event
ordering" of SURVEY §5 (race detection), run on the host before anything touches a GPU.

:func:`validate_programs` returns a list of violations (empty = valid):

* **dataflow** — every input of a kernel group is an external input, produced earlier on
  the same rank, or received (``recv``) earlier; a ``send`` only ships a produced tensor;
* **parameters** — every parameter group a kernel reads is resident (loaded or resident at
  a warm start, not evicted) when the group runs, and a warm-started program ends in the
  state it started from;
* **p2p pairing** — for each ordered pair of ranks the sequence of ``send(t, dst)`` /
  ``psend(group, dst)`` on the source equals the sequence of ``recv(t, src)`` / peer loads on
  the destination (RCCL p2p matches by order, there are no tags); a psend's group is resident
  at the offset it sends from, and no load overwrites it before the send is waited;
* **deadlock freedom** — a simulation of all ranks with non-blocking sends and blocking
  receives (the executor's isend/irecv + wait-at-use) runs every program to completion;
  a send the executor completes before reusing its buffer (``Instr.wait_sends``) blocks
  its rank until the receiver has posted the matching recv (rendezvous);
* **memory** — no two activations whose live ranges intersect share bytes of the
  activation arena, no ``run`` or ``recv`` writes bytes an in-flight ``send`` still reads
  unless it waits for that send first, no two resident parameter groups share bytes of
  the parameter arena, and everything stays inside the arena sizes the executor allocates.
"""
from __future__ import annotations

from collections import defaultdict, deque
from typing import Dict, List, Sequence, Tuple

from ..core.task import Task
from .program import Program


def _overlap(a: Tuple[int, int], b: Tuple[int, int]) -> bool:
    return a[0] < b[1] and b[0] < a[1]


def validate_programs(tasks: Sequence[Task], programs: Sequence[Program],
                      param_bytes: Dict[str, int]) -> List[str]:
    tmap = {t.id: t for t in tasks}
    errs: List[str] = []
    sends: Dict[Tuple[int, int], List[str]] = defaultdict(list)
    recvs: Dict[Tuple[int, int], List[str]] = defaultdict(list)

    for prog in programs:
        r = prog.rank
        have = set()
        resident: Dict[str, Tuple[int, int]] = {pid: (off, off + param_bytes.get(pid, 0))
                                                for pid, off in prog.start_resident.items()}
        act_live: Dict[str, Tuple[int, int, int]] = {}  # tid -> (lo, hi, last use index)
        inflight: Dict[int, Tuple[int, int]] = {}  # send index -> buffer region, until waited
        pinflight: Dict[int, Tuple[int, int]] = {}  # psend index -> parameter region, until waited
        last_use: Dict[str, int] = {}
        together, later, span_end = _coruns(prog)
        for i, ins in enumerate(prog.instrs):
            if ins.op == "run":
                for tid in ins.group:
                    for d in tmap[tid].dependencies:
                        last_use[d] = max(last_use.get(d, i), span_end.get(i, i))
            elif ins.op in ("send", "recv"):
                last_use[ins.task] = max(last_use.get(ins.task, i), i)
        for i, ins0 in enumerate(prog.instrs):
            if i in later:  # issued with its co-run span's first run
                continue
            for k in together.get(i, [i]):
                ins = prog.instrs[k]
                where = f"rank {r} instr {k} ({ins.op} {ins.task or ins.param})"
                _check_instr(k, ins, where, r, prog, tmap, param_bytes, errs, sends, recvs, have, resident,
                             act_live, inflight, pinflight, last_use, i)
        if prog.start_resident:
            end = {pid: reg[0] for pid, reg in resident.items()}
            if end != prog.start_resident:
                errs.append(f"rank {r}: warm-started program does not restore its start state "
                            f"({sorted(set(end.items()) ^ set(prog.start_resident.items()))[:4]}...)")
    # p2p pairing
    for key in set(sends) | set(recvs):
        if sends.get(key, []) != recvs.get(key, []):
            errs.append(f"p2p {key[0]}->{key[1]}: send order {sends.get(key, [])[:6]}... != recv order "
                        f"{recvs.get(key, [])[:6]}...")
    if not errs:
        errs.extend(_deadlock_check(programs))
    return errs


def _coruns(prog: Program):
    """Co-run spans (program.plan_coruns) as instruction indices: first run -> the span's
    parameter loads and members (all take effect there), the later ones, each member's span end."""
    run_at = {ins.task: i for i, ins in enumerate(prog.instrs) if ins.op == "run"}
    together: Dict[int, List[int]] = {}
    later: set = set()
    span_end: Dict[int, int] = {}
    for span in getattr(prog, "coruns", ()):
        idx = [run_at[t] for t in span]
        loads = [k for k in range(idx[0], idx[-1]) if prog.instrs[k].op == "load"]  # mapped up front
        together[idx[0]] = loads + idx
        later |= set(loads) | set(idx[1:])
        for k in idx:
            span_end[k] = idx[-1]
    return together, later, span_end


def _check_instr(i, ins, where, r, prog, tmap, param_bytes, errs, sends, recvs, have, resident, act_live, inflight,
                 pinflight, last_use, at) -> None:
    """One instruction of validate_programs (``at``: where it takes effect — a co-run span's
    member writes its output at the span's first run)."""
    if ins.op == "psend":
        if ins.param not in resident:
            errs.append(f"{where}: sends parameter group {ins.param} it does not hold")
        elif resident[ins.param][0] != ins.param_off:
            errs.append(f"{where}: psend offset {ins.param_off} != resident offset {resident[ins.param][0]}")
        sends[(r, ins.peer)].append(("param", ins.param))
        pinflight[i] = (ins.param_off, ins.param_off + param_bytes.get(ins.param, 0))
        return
    if ins.op == "load":
        off = prog.param_offset.get((i, ins.param))
        if off is None:
            errs.append(f"{where}: no arena offset for the load")
            return
        reg = (off, off + param_bytes.get(ins.param, 0))
        if ins.peer >= 0:
            recvs[(ins.peer, r)].append(("param", ins.param))
        for j in ins.wait_sends:
            pinflight.pop(j, None)
        for j, preg in pinflight.items():
            if _overlap(reg, preg):
                errs.append(f"{where}: overwrites the region of in-flight parameter send {j} without waiting")
        if reg[1] > prog.param_arena_bytes:
            errs.append(f"{where}: parameter region {reg} exceeds the arena ({prog.param_arena_bytes} B)")
        for pid, other in resident.items():
            if pid != ins.param and _overlap(reg, other):
                errs.append(f"{where}: overlaps resident parameter group {pid}")
        resident[ins.param] = reg
        return
    elif ins.op == "evict":
        if ins.param not in resident:
            errs.append(f"{where}: evicting a group that is not resident")
        resident.pop(ins.param, None)
    elif ins.op == "recv":
        sends_key = (ins.peer, r)
        recvs[sends_key].append(ins.task)
        have.add(ins.task)
    elif ins.op == "send":
        if ins.task not in have:
            errs.append(f"{where}: sends a tensor not produced/received on this rank")
        sends[(r, ins.peer)].append(ins.task)
        if ins.task in prog.act_offset:
            lo = prog.act_offset[ins.task]
            inflight[i] = (lo, lo + prog.act_bytes[ins.task])
    elif ins.op == "run":
        group = set(ins.group)
        for tid in ins.group:
            t = tmap[tid]
            for d in t.dependencies:
                if d in tmap and d not in have and d not in group:
                    errs.append(f"{where}: input {d} of {tid} is not available")
            for pid in t.params_needed:
                if pid not in resident:
                    errs.append(f"{where}: parameter group {pid} of {tid} is not resident")
            have.add(tid)
    # activation regions: define at run/recv, live until the last use
    if ins.op in ("run", "recv") and ins.task in prog.act_offset:
        lo = prog.act_offset[ins.task]
        hi = lo + prog.act_bytes[ins.task]
        for j in ins.wait_sends:
            inflight.pop(j, None)
        for j, reg in inflight.items():
            if _overlap((lo, hi), reg):
                errs.append(f"{where}: writes the buffer of in-flight send {j} "
                            f"({prog.instrs[j].task}->gpu{prog.instrs[j].peer}) without waiting for it")
        if hi > prog.act_arena_bytes:
            errs.append(f"{where}: activation region [{lo},{hi}) exceeds the arena ({prog.act_arena_bytes} B)")
        for other, (olo, ohi, oend) in act_live.items():
            if oend >= at and _overlap((lo, hi), (olo, ohi)):
                errs.append(f"{where}: output {ins.task} overwrites live activation {other}")
        act_live[ins.task] = (lo, hi, last_use.get(ins.task, len(prog.instrs)))


def _deadlock_check(programs: Sequence[Program]) -> List[str]:
    """Run all programs: a send is posted into a per-pair FIFO without blocking, a recv
    blocks until the matching message is at the head of its FIFO, and an instruction with
    ``wait_sends`` blocks until each of those sends has been taken by its receiver."""
    pc = [0] * len(programs)
    fifo: Dict[Tuple[int, int], deque] = defaultdict(deque)
    taken = set()  # (rank, send index) whose matching recv has been posted
    progress = True
    while progress:
        progress = False
        for prog in programs:
            r = prog.rank
            together = _coruns(prog)[0]
            while pc[r] < len(prog.instrs):
                ins = prog.instrs[pc[r]]
                waits = [j for k in together.get(pc[r], [pc[r]]) for j in prog.instrs[k].wait_sends]
                if any((r, j) not in taken for j in waits):
                    break
                is_precv = ins.op == "load" and ins.peer >= 0
                if ins.op in ("send", "psend"):
                    msg = ins.task if ins.op == "send" else ("param", ins.param)
                    fifo[(r, ins.peer)].append((msg, pc[r]))
                elif ins.op == "recv" or is_precv:
                    msg = ins.task if ins.op == "recv" else ("param", ins.param)
                    q = fifo[(ins.peer, r)]
                    if not q:
                        break
                    if q[0][0] != msg:
                        return [f"rank {r}: recv {msg} from {ins.peer} but the next message is {q[0][0]}"]
                    taken.add((ins.peer, q.popleft()[1]))
                pc[r] += 1
                progress = True
    stuck = [(p.rank, pc[p.rank]) for p in programs if pc[p.rank] < len(p.instrs)]
    if stuck:
        return [f"deadlock: ranks blocked at {stuck}"]
    return []


def device_deadlock_check(tasks: Sequence[Task], programs: Sequence[Program], eager: bool = True,
                          batched: bool = False, gpu: bool = True, routed: bool = True) -> List[str]:
    """Deadlock freedom under the DEVICE transport's progress rules (parallel/devp2p.py), which
    differ from RCCL's: a send completes when the consumer has PULLED it (its ack), not when the
    receive was posted, and an expert-parallel receive is pulled only once the device-side routing
    it needs is on the consumer — an expert's output at its post, a hidden state right after its
    router logits (DAGExecutor._plan_routed_edges). Each rank's stream runs its program in
    order: notifies never block, a pull waits for the producer's notify, and a write listed with
    ``wait_sends`` (a co-run span's first run: every member's) waits for those sends' acks.
    ``eager=False`` models pulling every routed receive at its first consumer instead (what the
    transport did before; a layer-major expert-parallel plan deadlocks under it). ``batched``
    models one wait for ALL of a program point's flags before any of its copies — fewer graph
    nodes, but an ack then waits for flags of other producers, and the 4-rank config-5 plan
    deadlocks under it: the executor pulls each receive after its own flag only. ``gpu`` /
    ``routed``: the executor's conditions for routed pulls (a whole-layer expert batch on the
    GPU pulls its tokens whole; DLS_EP_ROUTED=0 pulls everything whole at its post) — the rule
    itself is program.device_routed_edges, shared with the executor."""
    from .executor import MOE_BATCH
    from .program import device_routed_edges, moe_batched_ids

    tmap = {t.id: t for t in tasks}
    acts: List[List[Tuple[str, tuple, int]]] = []
    for prog in programs:
        r = prog.rank
        users: Dict[str, List[Task]] = defaultdict(list)
        at: Dict[str, int] = {}
        for i, ins in enumerate(prog.instrs):
            if ins.op == "run":
                for tid in ins.group:
                    at.setdefault(tid, i)
                    for d in tmap[tid].dependencies:
                        users[d].append(tmap[tid])
            elif ins.op == "recv":
                at.setdefault(ins.task, i)
        pull_at: Dict[int, List[str]] = defaultdict(list)
        out_rows = set()
        if routed:
            bat = moe_batched_ids(prog, tmap) if (gpu and MOE_BATCH) else set()
            routed_in, out_rows = device_routed_edges(prog, tmap, bat)
            for x, us in routed_in.items():
                pull_at[max(at[x], at.get(us[0].op.inputs[1], 0))].append(x)
        if not eager:  # every routed receive pulled right before its first consumer runs
            first = {x: min(at[u.id] for u in users[x]) for v in pull_at.values() for x in v}
            first.update({x: min(at[u.id] for u in users[x]) for x in out_rows})
            pull_at = defaultdict(list)
            for x, i in first.items():
                pull_at[i - 1].append(x)
        together, later, _ = _coruns(prog)
        deferred: Dict[str, tuple] = {}
        send_key: Dict[int, tuple] = {}
        a: List[Tuple[str, tuple, int]] = []
        ins_ = prog.instrs
        i = 0
        while i < len(ins_):
            ins = ins_[i]
            if ins.op in ("send", "recv"):
                # one p2p group, as DAGExecutor._post_p2p posts it: each receive's own send waits,
                # every notify, then each receive in order pulled after its own flag (an expert's
                # output rows too), each followed by the hidden states its router logits unlock
                j = i
                while j + 1 < len(ins_) and ins_[j + 1].op in ("send", "recv") \
                        and not any(i <= w <= j for w in ins_[j + 1].wait_sends):
                    j += 1
                pulls = []
                for k in range(i, j + 1):
                    x = ins_[k]
                    if x.op == "recv":
                        a.extend(("ack", send_key[w], k) for w in x.wait_sends if w in send_key)
                for k in range(i, j + 1):
                    x = ins_[k]
                    if x.op == "send":
                        send_key[k] = (r, x.peer, ("act", x.task))
                        a.append(("notify", send_key[k], k))
                due = []
                for k in range(i, j + 1):
                    x = ins_[k]
                    if x.op != "recv":
                        continue
                    key = (x.peer, r, ("act", x.task))
                    if any(x.task in v for v in pull_at.values()):
                        deferred[x.task] = key
                    else:
                        pulls.append(key)
                    now = [deferred.pop(h) for h in pull_at.get(k, []) if h in deferred]
                    if batched:
                        due += now
                    else:
                        a.extend(("pull", (key2,), k) for key2 in pulls + now)
                        pulls = []
                if batched:
                    a.extend(("pull", tuple(b), j) for b in (pulls, due) if b)
                i = j + 1
                continue
            waits = [w for k in together.get(i, [i]) for w in ins_[k].wait_sends] if i not in later else []
            if ins.op in ("run", "load"):
                a.extend(("ack", send_key[w], i) for w in waits if w in send_key)
            if ins.op == "psend":
                send_key[i] = (r, ins.peer, ("param", ins.param, ins.gpos))
                a.append(("notify", send_key[i], i))
            elif ins.op == "load" and ins.peer >= 0:
                a.append(("pull", ((ins.peer, r, ("param", ins.param, ins.gpos)),), i))
            due = [deferred.pop(h) for h in pull_at.get(i, []) if h in deferred]
            if due and batched:
                a.append(("pull", tuple(due), i))
            else:
                a.extend(("pull", (key,), i) for key in due)
            i += 1
        a.extend(("pull", (key,), -1) for key in deferred.values())
        a.extend(("ack", key, -1) for key in send_key.values())
        acts.append(a)
    ready, acked = set(), set()
    pc = [0] * len(programs)
    progress = True
    while progress:
        progress = False
        for k, prog in enumerate(programs):
            while pc[k] < len(acts[k]):
                kind, key, _ = acts[k][pc[k]]
                if kind == "notify":
                    ready.add(key)
                elif kind == "pull":  # a batch: every flag before any copy (and its ack)
                    if any(k2 not in ready for k2 in key):
                        break
                    acked.update(key)
                elif key not in acked:
                    break
                pc[k] += 1
                progress = True
    stuck = [(prog.rank, acts[k][pc[k]][0], acts[k][pc[k]][1], acts[k][pc[k]][2])
             for k, prog in enumerate(programs) if pc[k] < len(acts[k])]
    return [f"device transport deadlock: ranks blocked at {stuck[:4]}"] if stuck else []


def check_plan(p, device: bool = False, gpu: bool = True) -> List[str]:
    """validate_programs on a runtime.Plan; ``device``: plus the device transport's progress
    rules (for a plan that will run on that transport)."""
    errs = validate_programs(p.tasks, p.programs, p.param_bytes)
    if not errs and device:
        from .executor import EP_ROUTED

        errs = device_deadlock_check(p.tasks, p.programs, gpu=gpu, routed=EP_ROUTED)
    return errs
