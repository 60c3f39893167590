"""Device-initiated p2p transport: DAG edges moved by KERNELS on the ranks' own streams.

RCCL's send / recv are host-issued operations the executor cannot capture, so a multi-GPU step
is cut into hipGraph segments at every receive and replayed by the native runner (≈10-16 µs of
host time per segment). Here every edge is three small kernels instead (csrc/kernels/
p2p_device.hpp):

  producer P, after the producing kernel:  notify  — ready[slot] on the consumer := step
  consumer C, before the first consumer:   pull    — wait ready[slot] >= step, copy P's region
                                                     into C's (over xGMI when P is another GPU),
                                                     then ack[slot] on P := step
  P, before its region is written again:   wait    — ack[slot] >= step

plus one ``tick`` per step that bumps the rank's step counter, so a rank's WHOLE step — kernels
and edges — captures into ONE hipGraph and replays with fresh sequence numbers. Nothing pairs
transfers on the host: a message's slot is a pure function of the plan (:func:`edge_slots`),
the source address of a pull is the producer's arena base plus the offset its program gives
the region, and the flags live in each rank's mailbox (uncached device memory).

Ranks sharing a process (the single-GPU harness, parallel/loopback.py ``transport="device"``)
address each other's arenas directly; separate processes exchange IPC handles of their arenas
and mailboxes once (:meth:`DeviceP2PWorld.exchange`). A wait that does not see its flag within
``DLS_P2P_TIMEOUT_S`` sets the rank's error word and gives up — wrong numbers, never a hung
GPU; :meth:`DeviceComm.errors` reads it.

Ordering matches RCCL's p2p contract (the programs validated for it need nothing new): a send
never blocks (notify is a flag store); a receive is pulled where it is posted — at the
producer's position in the consumer's program, as an RCCL receive completes once both ends have
posted (pulling later, at the consumer, can deadlock: the producer may wait to reuse the region
for something the consumer needs first); a sent region is written again only after its
consumer pulled it. Routed expert-parallel rows are the exception: they are pulled by the
consumer's MoE code once the routing is known on the device, right after the receive.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import lifetime

TIMEOUT_S = float(os.environ.get("DLS_P2P_TIMEOUT_S", "10"))
_TICKS = int(TIMEOUT_S * 1e8)  # wall_clock64 runs at 100 MHz
ERR_PULL, ERR_ACK = 1, 2
BATCH = 16  # kP2PBatch (p2p_device.hpp): flags per batched notify launch
# fault injection for negative controls ONLY: message slots whose producer never notifies (the
# consumer's pull then times out into the error word and the executor raises TransportError)
DROP_NOTIFY = frozenset(int(v) for v in os.environ.get("DLS_P2P_DROP_NOTIFY", "").split(",") if v.strip())


def stalled_edges(slots, rank: int, step: int, ready, ack) -> List[str]:
    """The messages of ``rank`` still behind at ``step``: receives whose producer's notify has
    not arrived (ready[slot] < step) and sends whose consumer has not pulled (ack[slot] < step)."""
    out = []
    for (src, dst, key), slot in slots.items():
        what = "/".join(str(k) for k in key[1:])
        if dst == rank and ready[slot] < step:
            out.append(f"receive of {what} from rank {src} (slot {slot}): producer's notify not seen")
        elif src == rank and ack[slot] < step:
            out.append(f"send of {what} to rank {dst} (slot {slot}): consumer has not pulled it")
    return out


def edge_slots(programs) -> Dict[Tuple[int, int, tuple], int]:
    """Slot of every cross-rank message of a step, from the programs alone (the same on every
    rank): key (src rank, dst rank, what), what = ("act", task) for a DAG edge or ("param",
    group, gpos) for a parameter group filled from a peer (program.plan_peer_fills)."""
    slots: Dict[Tuple[int, int, tuple], int] = {}
    for pr in programs:
        for ins in pr.instrs:
            if ins.op == "send":
                key = (pr.rank, ins.peer, ("act", ins.task))
            elif ins.op == "psend":
                key = (pr.rank, ins.peer, ("param", ins.param, ins.gpos))
            else:
                continue
            if key in slots:
                raise ValueError(f"device p2p: message {key} sent twice in one step")
            slots[key] = len(slots)
    return slots


def source_regions(programs, param_bytes: Dict[str, int]) -> Dict[Tuple[int, int, tuple], Tuple[str, int, int]]:
    """Where each message's bytes sit on its producer: key -> (arena "act" | "param", offset,
    bytes) — the producer's program fixes every region, so a consumer computes its pull's
    source address from the producer's arena base alone."""
    out = {}
    for pr in programs:
        for ins in pr.instrs:
            if ins.op == "send":
                out[(pr.rank, ins.peer, ("act", ins.task))] = ("act", pr.act_offset[ins.task], pr.act_bytes[ins.task])
            elif ins.op == "psend":
                out[(pr.rank, ins.peer, ("param", ins.param, ins.gpos))] = (
                    "param", ins.param_off, int(param_bytes.get(ins.param, 0)))
    return out


class Mailbox:
    """One rank's flags: int64 [step, bytes pulled, ready[S], ack[S]], int32 tickets[S] and an
    error word, in uncached device memory (polled by one lane, written by peers)."""

    def __init__(self, n_slots: int, device):
        from .. import ops

        self.S = n_slots
        n64 = 2 + 2 * n_slots
        n32 = n_slots + 1
        nbytes = (n64 * 8 + n32 * 4 + 255) // 256 * 256
        self.raw = lifetime.keep(self, ops.ext().alloc_device(nbytes, 3))  # hipDeviceMallocUncached
        self.raw.zero_()
        i64 = self.raw[:n64 * 8].view(torch.int64)
        i32 = self.raw[n64 * 8:n64 * 8 + n32 * 4].view(torch.int32)
        self.step = i64[0:1]
        self.moved = i64[1:2]
        self.ready = i64[2:2 + n_slots]
        self.ack = i64[2 + n_slots:2 + 2 * n_slots]
        self.tickets = i32[:n_slots]
        self.err = i32[n_slots:n_slots + 1]
        self.base = self.raw.data_ptr()

    def ready_addr(self, base: int, slot: int) -> int:
        return base + 8 * (2 + slot)

    def ack_addr(self, base: int, slot: int) -> int:
        return base + 8 * (2 + self.S + slot)


class DeviceP2PWorld:
    """The transport state a job shares: message slots, source regions and every rank's
    addresses (arena bases, mailbox). ``local_ranks``: the ranks living in this process (all of
    them for the single-GPU harness, one for a process-per-GPU job)."""

    def __init__(self, plan, device, local_ranks: Sequence[int], delay_us: float = 0.0, poison: bool = False):
        self.world = plan.world
        self.device = torch.device(device)
        self.slots = edge_slots(plan.programs)
        self.sources = source_regions(plan.programs, plan.param_bytes)
        self.delay_us, self.poison = float(delay_us), bool(poison)
        self.mail = {r: Mailbox(len(self.slots), self.device) for r in local_ranks}
        self.bases: Dict[int, Dict[str, int]] = {}  # rank -> {"act", "param", "mail"} addresses here
        self._opened: List[int] = []
        self._exported: Dict[int, Dict[str, torch.Tensor]] = {}

    def attach(self, rank: int, act: torch.Tensor, param: torch.Tensor) -> None:
        self.bases[rank] = {"act": act.data_ptr(), "param": param.data_ptr(), "mail": self.mail[rank].base}
        self._exported[rank] = {"act": act, "param": param, "mail": self.mail[rank].raw}

    def exchange(self, pg) -> None:
        """Process-per-GPU job: publish this process's arenas and mailbox as IPC handles and open
        every peer's (one collective, at executor construction)."""
        import torch.distributed as dist

        from .. import ops

        e = ops.ext()
        mine = {r: {k: e.ipc_handle(t) for k, t in d.items()} for r, d in self._exported.items()}
        allh: List[Optional[dict]] = [None] * dist.get_world_size(pg)
        dist.all_gather_object(allh, mine, group=pg)
        for d in allh:
            for r, hs in (d or {}).items():
                if r in self.bases:
                    continue
                addr = {}
                for k, (h, off) in hs.items():
                    base = e.ipc_open(h)
                    self._opened.append(base)
                    addr[k] = base + off
                self.bases[r] = addr

    def close(self) -> None:
        from .. import ops

        for b in self._opened:
            try:
                ops.ext().ipc_close(b)
            except RuntimeError:
                pass
        self._opened = []


class DeviceP2PGroup:
    """What a rank's executor gets as ``pg`` for the device transport."""

    def __init__(self, world: DeviceP2PWorld, rank: int, pg=None):
        self.world, self.rank, self.pg = world, rank, pg

    def size(self) -> int:
        return self.world.world


class _SendWork:
    __slots__ = ("comm", "slot", "done")

    def __init__(self, comm, slot: int):
        self.comm, self.slot, self.done = comm, slot, False

    def wait(self):
        if not self.done:
            self.done = True
            m = self.comm.mb
            self.comm.e.p2p_wait(m.ack[self.slot:self.slot + 1], m.step, m.err, _TICKS, ERR_ACK)


class _RecvWork:
    __slots__ = ("comm", "slot", "buf", "src", "done")

    def __init__(self, comm, slot: int, buf: torch.Tensor, src: Tuple[int, str, int]):
        self.comm, self.slot, self.buf, self.src, self.done = comm, slot, buf, src, False

    def _args(self):
        c = self.comm
        peer, arena, off = self.src
        pb = c.w.bases[peer]
        m = c.mb
        return (pb[arena] + off, m.ready[self.slot:self.slot + 1], m.ack_addr(pb["mail"], self.slot),
                m.tickets[self.slot:self.slot + 1])

    def wait(self):
        """Pull the whole region (the receiving rank's stream; later kernels see it)."""
        if not self.done:
            self.done = True
            src, ready, ack, ticket = self._args()
            m = self.comm.mb
            self.comm.e.p2p_pull(src, self.buf, ready, ack, ticket, m.step, m.err, _TICKS, m.moved)

    def pull_rows(self, dst: torch.Tensor, row_bytes: int, idx: Optional[torch.Tensor], off: torch.Tensor,
                  experts: torch.Tensor, max_rows: int) -> None:
        """Pull only routed rows instead (expert parallelism, the device-side routing ``off`` /
        ``idx`` decides which): for each expert in ``experts``, rows [off[e], off[e+1]) of the
        expert-sorted order — gathered from source rows ``idx[j]`` into dst row j, or (``idx``
        None) compact rows 0.. of the source into the same rows of ``dst``."""
        if self.done:
            return
        self.done = True
        src, ready, ack, ticket = self._args()
        m = self.comm.mb
        self.comm.e.p2p_pull_rows(src, dst, int(row_bytes), idx, off, experts, int(max_rows), ready, ack, ticket,
                                  m.step, m.err, _TICKS, m.moved)


class _NoWork:
    def wait(self):
        pass

    def pull_rows(self, *a, **k):
        pass


class DeviceComm:
    kind = "device"

    def __init__(self, group: DeviceP2PGroup):
        from .. import ops

        self.w = group.world
        self.rank = group.rank
        self.pg = group.pg
        self.mb = self.w.mail[self.rank]
        self.e = ops.ext()
        # a DRY step posts nothing and waits for nothing (no tick either, on every rank alike):
        # the single-GPU harness runs one per rank, one rank at a time, before the real steps, so
        # a rank's first-step allocations — which may synchronise the whole device — never wait
        # behind a peer rank's spinning pull in the same process
        self.dry = False

    def attach(self, ex) -> None:
        """Register the executor's arenas (their base addresses are what peers pull from)."""
        self.w.attach(self.rank, ex.act_slab, ex.param_slab)
        if self.pg is not None:
            self.w.exchange(self.pg)

    def begin_step(self) -> None:
        if not self.dry:
            self.e.p2p_tick(self.mb.step)

    def _slot(self, src: int, dst: int, key) -> int:
        try:
            return self.w.slots[(src, dst, key)]
        except KeyError:
            raise RuntimeError(f"device p2p: no message {key} from rank {src} to rank {dst} in the plan") from None

    def isend(self, buf: torch.Tensor, peer: int, key=None):
        slot = self._slot(self.rank, peer, key)
        if self.dry:
            return _NoWork()
        if self.w.delay_us > 0:  # single-GPU harness: the notify lands late (a missing wait shows)
            self.e.p2p_delay(self.w.delay_us, self.mb.step)
        if slot not in DROP_NOTIFY:
            self.e.p2p_notify(self.mb.ready_addr(self.w.bases[peer]["mail"], slot), self.mb.step)
        return _SendWork(self, slot)

    def irecv(self, buf: torch.Tensor, peer: int, key=None):
        slot = self._slot(peer, self.rank, key)
        arena, off, nbytes = self.w.sources[(peer, self.rank, key)]
        # ``buf``: the receiver's whole region for the message (uint8, as its program sized it)
        region = buf.view(torch.uint8) if buf.is_contiguous() and buf.dim() == 1 else None
        if region is None or region.numel() != nbytes:
            raise RuntimeError(f"device p2p: receive region of {key} does not match the producer's "
                               f"({None if region is None else region.numel()} vs {nbytes} bytes)")
        if self.dry:
            return _NoWork()
        if self.w.poison:
            region.fill_(0xFF)  # bf16 NaN until the pull lands
        return _RecvWork(self, slot, region, (peer, arena, off))

    def batch(self, ops_: Sequence[Tuple[bool, torch.Tensor, int, object]]) -> List[object]:
        """One program point's sends and receives; two or more sends notify from ONE launch (a
        notify never waits). Receives are pulled one by one, each after its own flag: one wait for
        all of a point's flags would make an ack wait for other producers (validate.py,
        ``device_deadlock_check(batched=True)``)."""
        sends = [k for k, (snd, _, _, _) in enumerate(ops_) if snd]
        if len(sends) < 2 or self.dry:
            return [self.isend(b, p, k) if snd else self.irecv(b, p, k) for snd, b, p, k in ops_]
        out: List[object] = [None if snd else self.irecv(b, p, k) for snd, b, p, k in ops_]
        slots = {k: self._slot(self.rank, ops_[k][2], ops_[k][3]) for k in sends}
        if self.w.delay_us > 0:
            self.e.p2p_delay(self.w.delay_us, self.mb.step)
        flags = [self.mb.ready_addr(self.w.bases[ops_[k][2]]["mail"], slots[k]) for k in sends
                 if slots[k] not in DROP_NOTIFY]
        for i in range(0, len(flags), BATCH):
            self.e.p2p_notify_many(flags[i:i + BATCH], self.mb.step)
        for k in sends:
            out[k] = _SendWork(self, slots[k])
        return out

    def reset_errors(self) -> None:
        """Clear the error word (after warm-up: a first step's lazy code-object loading on one
        rank can outlast a peer's wait; sequence numbers are monotonic, so the protocol itself
        recovers on the next step)."""
        self.mb.err.zero_()

    def bytes_pulled(self) -> int:
        """Bytes this rank pulled from its peers since the mailbox was made (host read)."""
        return int(self.mb.moved.item())

    def errors(self) -> int:
        """The rank's error word (host read: synchronises): bit 0 a pull, bit 1 an ack wait
        timed out."""
        return int(self.mb.err.item())

    def stalled(self) -> List[str]:
        """This rank's messages still behind its step counter (host reads: synchronises)."""
        return stalled_edges(self.w.slots, self.rank, int(self.mb.step.item()), self.mb.ready.tolist(),
                             self.mb.ack.tolist())


# ---------------------------------------------------------------------------------------------
# The same protocol on the HOST (CPU tensors, every rank a thread of one process): one flag per
# message slot and step number, a pull that waits for its producer's notify, a send whose
# completion is the consumer's pull (its ack) — with a condition variable where the GPU spins.
# The executor takes the device transport's code paths unchanged (regions pulled at their post,
# routed expert rows pulled once their routing is on the rank, co-run expert batches), so the CPU
# suite exercises them; a progress error (a send waiting for a pull that comes later) shows up
# as a wait that times out, and the error word records it as on the GPU.


class HostP2PWorld:
    """Slots, source regions and every rank's flags and arenas of a job whose ranks are threads
    of this process (parallel/loopback.py, ``transport="device"`` on the CPU)."""

    def __init__(self, plan, local_ranks: Sequence[int], poison: bool = False, timeout_s: float = 30.0):
        import threading

        self.world = plan.world
        self.slots = edge_slots(plan.programs)
        self.sources = source_regions(plan.programs, plan.param_bytes)
        self.poison, self.timeout_s = bool(poison), float(timeout_s)
        S = len(self.slots)
        self.cv = threading.Condition()
        self.ready = {r: [0] * S for r in local_ranks}
        self.ack = {r: [0] * S for r in local_ranks}
        self.step = {r: 0 for r in local_ranks}
        self.err = {r: 0 for r in local_ranks}
        self.moved = {r: 0 for r in local_ranks}
        self.aborted = False
        self.arenas: Dict[int, Dict[str, torch.Tensor]] = {}

    def attach(self, rank: int, act: torch.Tensor, param: torch.Tensor) -> None:
        self.arenas[rank] = {"act": act.view(-1).view(torch.uint8), "param": param.view(-1).view(torch.uint8)}

    def wait_for(self, pred, rank: int, code: int) -> bool:
        """Block until ``pred()`` (under the condition's lock); on timeout — or once a rank of
        the job has failed (:meth:`abort`) — fold ``code`` into the rank's error word and give
        up (wrong numbers, as on the GPU, never a hang)."""
        with self.cv:
            if self.cv.wait_for(lambda: pred() or self.aborted, self.timeout_s) and not self.aborted:
                return True
            if pred():
                return True
            self.err[rank] |= code
            # the job's protocol is broken from here on: later waits give up at once (a second
            # full timeout per wait would only delay the failure the executor now reports)
            self.aborted = True
            self.cv.notify_all()
            return False

    def abort(self) -> None:
        """A rank of the job failed: every wait still pending (or posted later) gives up at
        once instead of after its full timeout."""
        with self.cv:
            self.aborted = True
            self.cv.notify_all()

    def close(self) -> None:
        pass


class HostP2PGroup:
    def __init__(self, world: HostP2PWorld, rank: int):
        self.world, self.rank = world, rank

    def size(self) -> int:
        return self.world.world


class _HostSend:
    __slots__ = ("comm", "slot", "step", "done")

    def __init__(self, comm, slot: int, step: int):
        self.comm, self.slot, self.step, self.done = comm, slot, step, False

    def wait(self):
        if not self.done:
            self.done = True
            w, r = self.comm.w, self.comm.rank
            w.wait_for(lambda: w.ack[r][self.slot] >= self.step, r, ERR_ACK)


class _HostRecv:
    __slots__ = ("comm", "slot", "buf", "src", "step", "done")

    def __init__(self, comm, slot: int, buf: torch.Tensor, src: Tuple[int, str, int], step: int):
        self.comm, self.slot, self.buf, self.src, self.step, self.done = comm, slot, buf, src, step, False

    def _arrived(self):
        w, r = self.comm.w, self.comm.rank
        ok = w.wait_for(lambda: w.ready[r][self.slot] >= self.step, r, ERR_PULL)
        peer, arena, off = self.src
        return ok, w.arenas[peer][arena][off:off + self.buf.numel()]

    def _acked(self, nbytes: int):
        w, r = self.comm.w, self.comm.rank
        with w.cv:
            w.ack[self.src[0]][self.slot] = max(w.ack[self.src[0]][self.slot], self.step)
            w.moved[r] += int(nbytes)
            w.cv.notify_all()

    def wait(self):
        """Pull the whole region."""
        if not self.done:
            self.done = True
            ok, src = self._arrived()
            if ok:
                self.buf.copy_(src)
            self._acked(self.buf.numel())

    def pull_rows(self, dst: torch.Tensor, row_bytes: int, idx: Optional[torch.Tensor], off: torch.Tensor,
                  experts: torch.Tensor, max_rows: int) -> None:
        """Routed rows only (the DeviceComm contract): for each listed expert, rows
        [off[e], off[e+1]) of the expert-sorted order — gathered through ``idx`` into the same
        rows of ``dst``, or (``idx`` None) compact rows 0.. of the source into rows 0.. of dst."""
        if self.done:
            return
        self.done = True
        ok, src = self._arrived()
        moved = 0
        if ok:
            s = src[:src.numel() // row_bytes * row_bytes].view(-1, row_bytes)
            d = dst.view(-1).view(torch.uint8)
            d = d[:d.numel() // row_bytes * row_bytes].view(-1, row_bytes)
            o = [int(v) for v in off.tolist()]
            for e in experts.tolist():
                lo, hi = o[e], o[e + 1]
                if hi <= lo:
                    continue
                if idx is not None:
                    d[lo:hi] = s[idx[lo:hi].long()]
                else:
                    d[:hi - lo] = s[:hi - lo]
                moved += (hi - lo) * row_bytes
        self._acked(moved)


class HostDeviceComm:
    """DeviceComm's contract on the host (see HostP2PWorld)."""
    kind = "device"

    def __init__(self, group: HostP2PGroup):
        self.w = group.world
        self.rank = group.rank
        self.dry = False

    def attach(self, ex) -> None:
        self.w.attach(self.rank, ex.act_slab, ex.param_slab)

    def begin_step(self) -> None:
        if not self.dry:
            with self.w.cv:
                self.w.step[self.rank] += 1

    def _slot(self, src: int, dst: int, key) -> int:
        try:
            return self.w.slots[(src, dst, key)]
        except KeyError:
            raise RuntimeError(f"device p2p: no message {key} from rank {src} to rank {dst} in the plan") from None

    def isend(self, buf: torch.Tensor, peer: int, key=None):
        slot = self._slot(self.rank, peer, key)
        if self.dry:
            return _NoWork()
        w = self.w
        with w.cv:
            step = w.step[self.rank]
            if slot not in DROP_NOTIFY:
                w.ready[peer][slot] = max(w.ready[peer][slot], step)
            w.cv.notify_all()
        return _HostSend(self, slot, step)

    def irecv(self, buf: torch.Tensor, peer: int, key=None):
        slot = self._slot(peer, self.rank, key)
        arena, off, nbytes = self.w.sources[(peer, self.rank, key)]
        region = buf.view(torch.uint8) if buf.is_contiguous() and buf.dim() == 1 else None
        if region is None or region.numel() != nbytes:
            raise RuntimeError(f"device p2p: receive region of {key} does not match the producer's "
                               f"({None if region is None else region.numel()} vs {nbytes} bytes)")
        if self.dry:
            return _NoWork()
        if self.w.poison:
            region.fill_(0xFF)  # bf16 NaN until the pull lands
        return _HostRecv(self, slot, region, (peer, arena, off), self.w.step[self.rank])

    def batch(self, ops_: Sequence[Tuple[bool, torch.Tensor, int, object]]) -> List[object]:
        return [self.isend(b, p, k) if s else self.irecv(b, p, k) for s, b, p, k in ops_]

    def reset_errors(self) -> None:
        self.w.err[self.rank] = 0

    def bytes_pulled(self) -> int:
        return self.w.moved[self.rank]

    def errors(self) -> int:
        return self.w.err[self.rank]

    def stalled(self) -> List[str]:
        w = self.w
        with w.cv:
            return stalled_edges(w.slots, self.rank, w.step[self.rank], w.ready[self.rank], w.ack[self.rank])
