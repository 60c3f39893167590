"""Point-to-point transport of one rank's executor.

The executor moves DAG edges with three primitives — post a send, post a receive, and wait for
a posted op (stream-side on a GPU: the caller's stream waits, the host does not) — plus a
*group* of such posts issued together (one ``ncclGroupStart/End`` through
``dist.batch_isend_irecv``).

Two transports implement them:

* :class:`DistComm` — ``torch.distributed`` (backend ``nccl`` = RCCL over xGMI on MI355X,
  ``gloo`` on the CPU test backend), one process per GPU;
* :class:`LoopComm` — the single-GPU loopback hub (``csrc/kernels/loopback.cpp``): several ranks
  in ONE process sharing one GPU, each on its own stream and host thread, transfers copied on
  the hub's stream behind a spinning delay kernel with poisoned receive buffers, so a missing
  stream wait shows up as NaN in the result (parallel/loopback.py).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


class _HubWork:
    __slots__ = ("hub", "op", "keep")

    def __init__(self, hub, op: int, keep=None):
        self.hub, self.op, self.keep = hub, op, keep

    def wait(self):
        if self.op is not None:
            self.hub.wait(self.op)
            self.op = None
            self.keep = None


class _GroupWork:
    """The one work of a coalesced group, handed to every op of the group (waiting for any op
    waits for the whole group, as with ncclGroupEnd)."""
    __slots__ = ("works",)

    def __init__(self, works):
        self.works = list(works)

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


class DistComm:
    kind = "dist"

    def __init__(self, pg):
        self.pg = pg

    def isend(self, buf: torch.Tensor, peer: int):
        return dist.isend(buf, dst=peer, group=self.pg)

    def irecv(self, buf: torch.Tensor, peer: int):
        return dist.irecv(buf, src=peer, group=self.pg)

    def batch(self, ops: Sequence[Tuple[bool, torch.Tensor, int]]) -> List[object]:
        """Post ``ops`` = [(is_send, buffer, peer)] as ONE group; returns a work per op."""
        if len(ops) == 1:
            s, b, p = ops[0]
            return [self.isend(b, p) if s else self.irecv(b, p)]
        p2p = [dist.P2POp(dist.isend if s else dist.irecv, b, p, group=self.pg) for s, b, p in ops]
        works = dist.batch_isend_irecv(p2p)
        if len(works) == len(ops):  # backend without coalescing (gloo): one work per op
            return works
        g = _GroupWork(works)  # RCCL: the group's single work
        return [g] * len(ops)


class LoopbackGroup:
    """What a loopback rank's executor gets as ``pg``: the shared hub, this rank, and the
    job-wide lock that makes a coalesced group's posts visible to the peers all at once."""

    def __init__(self, hub, rank: int, world: int, group_lock=None):
        import threading

        self.hub, self.rank, self.world = hub, rank, world
        self.group_lock = group_lock or threading.Lock()

    def size(self) -> int:
        return self.world


class LoopComm:
    kind = "loopback"

    def __init__(self, group: LoopbackGroup):
        self.g = group
        self.hub = group.hub
        self.rank = group.rank

    def isend(self, buf: torch.Tensor, peer: int):
        return _HubWork(self.hub, self.hub.post(True, buf, self.rank, peer), buf)

    def irecv(self, buf: torch.Tensor, peer: int):
        return _HubWork(self.hub, self.hub.post(False, buf, self.rank, peer), buf)

    def batch(self, ops: Sequence[Tuple[bool, torch.Tensor, int]]) -> List[object]:
        """ONE group, as ``ncclGroupStart/End``: every op of it is posted under the job-wide group
        lock, so no peer matches against a partly posted group (a peer's post sees all of the
        group's ops or none), and — as with RCCL's coalesced group — the group's single work
        completes when every op has: waiting for any op waits for the whole group."""
        if len(ops) == 1:
            s, b, p = ops[0]
            return [self.isend(b, p) if s else self.irecv(b, p)]
        with self.g.group_lock:
            works = [self.isend(b, p) if s else self.irecv(b, p) for s, b, p in ops]
        g = _GroupWork(works)
        return [g] * len(ops)


def init_world(rank: int, world: int, device=None) -> None:
    """``init_process_group`` for an executor job: ``nccl`` (= RCCL) bound to this rank's GPU
    with ``device_id`` (the communicator is created eagerly), ``gloo`` on the CPU; then one
    barrier on the whole group. Programs post each point's sends / receives as ONE
    ``batch_isend_irecv`` group, which torch documents as undefined when it is the group's first
    collective and not every rank takes part — the barrier makes sure it never is."""
    import torch
    import torch.distributed as dist

    gpu = device is not None and torch.device(device).type == "cuda"
    dist.init_process_group("nccl" if gpu else "gloo", rank=rank, world_size=world,
                            **({"device_id": torch.device(device)} if gpu else {}))
    dist.barrier()


def make_comm(pg):
    """The transport for an executor's ``pg`` argument (None: single rank, no p2p)."""
    if pg is None:
        return None
    if isinstance(pg, LoopbackGroup):
        return LoopComm(pg)
    from .devp2p import DeviceComm, DeviceP2PGroup, HostDeviceComm, HostP2PGroup

    if isinstance(pg, DeviceP2PGroup):
        return DeviceComm(pg)
    if isinstance(pg, HostP2PGroup):
        return HostDeviceComm(pg)
    return DistComm(pg)


def loopback_groups(world: int, delay_us: float = 20.0, poison: bool = True, timeout_s: float = 120.0):
    """One :class:`LoopbackGroup` per rank of a ``world``-rank job living in this process."""
    from .. import ops

    import threading

    hub = ops.ext().LoopbackHub(world, delay_us, poison, timeout_s)
    lock = threading.Lock()
    return [LoopbackGroup(hub, r, world, lock) for r in range(world)]
