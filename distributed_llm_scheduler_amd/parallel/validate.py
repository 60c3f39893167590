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
        for i, ins in enumerate(prog.instrs):
            if ins.op == "run":
                for tid in ins.group:
                    for d in tmap[tid].dependencies:
                        last_use[d] = i
            elif ins.op in ("send", "recv"):
                last_use[ins.task] = max(last_use.get(ins.task, i), i)
        for i, ins in enumerate(prog.instrs):
            where = f"rank {r} instr {i} ({ins.op} {ins.task or ins.param})"
            if ins.op == "psend":
                if ins.param not in resident:
                    errs.append(f"{where}: sends parameter group {ins.param} it does not hold")
                elif resident[ins.param][0] != ins.param_off:
                    errs.append(f"{where}: psend offset {ins.param_off} != resident offset {resident[ins.param][0]}")
                sends[(r, ins.peer)].append(("param", ins.param))
                pinflight[i] = (ins.param_off, ins.param_off + param_bytes.get(ins.param, 0))
                continue
            if ins.op == "load":
                off = prog.param_offset.get((i, ins.param))
                if off is None:
                    errs.append(f"{where}: no arena offset for the load")
                    continue
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
                    if oend >= i and _overlap((lo, hi), (olo, ohi)):
                        errs.append(f"{where}: output {ins.task} overwrites live activation {other}")
                act_live[ins.task] = (lo, hi, last_use.get(ins.task, len(prog.instrs)))
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
            while pc[r] < len(prog.instrs):
                ins = prog.instrs[pc[r]]
                if any((r, j) not in taken for j in ins.wait_sends):
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


def check_plan(p) -> List[str]:
    """validate_programs on a runtime.Plan."""
    return validate_programs(p.tasks, p.programs, p.param_bytes)
