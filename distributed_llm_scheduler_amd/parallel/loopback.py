"""Single-GPU multi-rank harness: a ``world``-rank job in ONE process on ONE device.

Every rank is a real :class:`DAGExecutor` with its own program, arenas, compute stream and host
thread; their DAG edges go through the loopback hub (``csrc/kernels/loopback.cpp``), which gives
the p2p primitives RCCL's semantics — posts ordered after the rank's enqueued kernels, the copy
on a separate stream, ``wait()`` making the consumer's stream wait — and adds two checks:

* every transfer runs behind a spinning delay kernel (``delay_us``), so the copy lands well after
  the consumer's next kernels would have started had they not been ordered after it;
* every receive buffer is filled with 0xFF (bf16 NaN) when the receive is posted (``poison``),
  so a consumer that reads it early computes NaN, and a producer that overwrites a buffer before
  its send completed sends the wrong bytes.

The same executor paths as a multi-process RCCL job run here — the eager Python issue loop,
segment hipGraphs around the p2p points, the native step runner's SEND / RECV / WORK_WAIT and
group actions, peer parameter fills — so a one-GPU box checks the multi-GPU path with real
device asynchrony (a gloo job cannot: its ``wait()`` blocks the host). CPU tensors work too
(copies at match time), for the CPU test suite.
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import torch

from .comm import loopback_groups


@dataclass
class LoopbackRun:
    executors: list
    stats: list                    # each rank's StepStats of its last step
    hub: object
    issue_modes: List[Optional[str]] = field(default_factory=list)
    step_ms: List[float] = field(default_factory=list)
    # host time per step.step() call (µs, mean over the timed steps): what issuing a step costs
    host_us: List[float] = field(default_factory=list)
    # device transport: each rank's error word after the warm-up steps (then cleared)
    warmup_errors: List[int] = field(default_factory=list)
    # expert-parallel capacity groups each rank widened after an overflow (then ran a step again)
    ep_widened: List[list] = field(default_factory=list)


def run_loopback(plan, device, steps: int = 3, warmup: int = 2, capture: bool = True, delay_us: float = 20.0,
                 poison: bool = True, store=None, timeout_s: float = 120.0,
                 before_steps: Optional[Callable] = None, cpu_runner: bool = False,
                 sync_debug: bool = False, autotune: bool = False, transport: str = "hub",
                 single_issue: bool = False, p2p_timeout_s: Optional[float] = None,
                 ep_exact: bool = True) -> LoopbackRun:
    """Build one executor per rank of ``plan`` on ``device``, then drive every rank from its own
    thread: ``warmup`` eager steps, capture (segment hipGraphs + native runner for programs with
    p2p), ``steps`` timed steps. ``before_steps(executors)`` may patch the executors first
    (negative controls). ``cpu_runner``: on the CPU backend, replay the steps from the native
    step runner (kernel groups as callbacks) instead of the Python issue loop. ``sync_debug``:
    the timed steps run under torch's sync debug mode "error" (any device->host synchronising
    call inside a step raises). ``autotune``: tune GEMM shapes missing from the table first (off:
    the kernel's heuristic config — the harness checks ordering and numerics, not speed).
    ``transport="device"``: the edges are moved by kernels (parallel/devp2p.py) — notify,
    pull and ack flags, no host pairing — and each rank's whole step captures into ONE hipGraph;
    ``delay_us`` then delays every notify and ``poison`` fills each receive region with NaN
    when the receive is posted (``p2p_timeout_s``: the host transport's wait limit on the CPU;
    on the GPU devp2p's DLS_P2P_TIMEOUT_S). ``ep_exact``: when an expert-parallel capacity edge
    overflowed in the steps, every rank widens its overflowed groups and the job runs one more
    step (``ep_widened``), so the outputs are exact. ``single_issue`` (captured whole-step graphs only): after
    warm-up, ONE host thread issues every rank's timed steps round-robin (graph launches are
    asynchronous), so ``host_us`` is the issue cost of a step without GIL contention between
    rank threads. On the CPU the same protocol runs with host waits (devp2p.HostP2PWorld)."""
    from . import lifetime

    with lifetime.quiesced():
        # garbage of earlier runs (executors, their hipGraphs / runners / buffers) is collected and
        # destroyed here, on the calling thread, and the cyclic collector stays paused while the
        # rank threads capture: a graph torn down by a finaliser on one rank thread while another
        # is inside a capture aborted the process (parallel/lifetime.py)
        return _run_loopback(plan, device, steps, warmup, capture, delay_us, poison, store, timeout_s,
                             before_steps, cpu_runner, sync_debug, autotune, transport, single_issue, p2p_timeout_s,
                             ep_exact)


def _run_loopback(plan, device, steps, warmup, capture, delay_us, poison, store, timeout_s, before_steps,
                  cpu_runner, sync_debug, autotune, transport, single_issue, p2p_timeout_s,
                  ep_exact) -> LoopbackRun:
    from . import executor as exm
    from . import runtime

    device = torch.device(device)
    gpu = device.type == "cuda"
    world = plan.world
    dw = None
    if transport == "device" and not gpu:
        # the device transport's protocol with host waits (devp2p.HostP2PWorld): the executor's
        # device-transport paths on the CPU, a progress error as a timed-out wait
        from .devp2p import HostP2PGroup, HostP2PWorld
        dw = HostP2PWorld(plan, range(world), poison=poison,
                          timeout_s=p2p_timeout_s if p2p_timeout_s is not None else min(timeout_s, 30.0))
        groups = [HostP2PGroup(dw, r) for r in range(world)]
    elif transport == "device":
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        if 4 * world > queues:
            # a pull / ack wait spins on its rank's stream; a peer's stream (compute, refill copy
            # or capture: up to 3 per rank, + the default) on the same hardware queue would be
            # queued behind it — every wait then times out (wrong numbers, never a hang)
            raise ValueError(f"device transport with {world} ranks in one process needs GPU_MAX_HW_QUEUES >= "
                             f"{4 * world} (set before the first CUDA call; it is {queues})")
        from .devp2p import DeviceP2PGroup, DeviceP2PWorld
        dw = DeviceP2PWorld(plan, device, range(world), delay_us=delay_us, poison=poison)
        groups = [DeviceP2PGroup(dw, r) for r in range(world)]
    elif transport == "hub":
        groups = loopback_groups(world, delay_us=delay_us if gpu else 0.0, poison=poison, timeout_s=timeout_s)
    else:
        raise ValueError(f"unknown transport {transport!r}")
    store = store or runtime.make_store(plan)
    # executors are built on this thread (autotuning and weight transforms are not thread-safe)
    if gpu and transport == "device":
        streams = _rank_streams(device, world)
    else:
        streams = [torch.cuda.Stream(device) for _ in range(world)] if gpu else [None] * world
    exs = []
    for r in range(world):
        if gpu:
            with torch.cuda.stream(streams[r]):
                exs.append(runtime.make_executor(plan, r, device, store, pg=groups[r], use_graph=capture,
                                                 autotune=autotune))
        else:
            exs.append(runtime.make_executor(plan, r, device, store, pg=groups[r], use_graph=False))
    if gpu:
        torch.cuda.synchronize(device)
    if transport == "device" and gpu:
        # one DRY step per rank, one rank at a time (no p2p, garbage numbers): first-step
        # allocations and weight transforms — some synchronise the whole device — happen before
        # any rank's kernels spin on a peer's flag in this shared process (a multi-process job
        # needs none: there a device-wide wait waits for that process's own streams only)
        for r, ex in enumerate(exs):
            ex.comm.dry = True
            with torch.cuda.stream(streams[r]):
                ex.step()
            ex.comm.dry = False
            streams[r].synchronize()
    if before_steps is not None:
        before_steps(exs)
    stats = [None] * world
    ms = [0.0] * world
    host_us = [0.0] * world
    warm_err = [0] * world
    errors = []
    start = threading.Barrier(world)

    def drive(r):
        import time

        try:
            if gpu:
                torch.cuda.set_device(device)
            ctx = torch.cuda.stream(streams[r]) if gpu else _Null()
            with ctx:
                ex = exs[r]
                for _ in range(warmup):
                    ex.step()
                # every rank's eager warm-up (first-step allocations and weight transforms) is
                # over before ANY rank starts capturing: nothing eager runs beside a capture
                start.wait()
                if capture and gpu:
                    ex.capture()
                if transport == "device":
                    if gpu:
                        streams[r].synchronize()
                    start.wait()  # every rank past its warm-up before any error word is cleared
                    warm_err[r] = ex.comm.errors()
                    ex.reset_transport_errors()
                elif cpu_runner and not gpu and not ex.build_runner():
                    raise RuntimeError("CPU step runner refused the program")
                start.wait()
                if sync_debug and gpu and r == 0:
                    torch.cuda.set_sync_debug_mode("error")
                start.wait()
                if single_issue:
                    return  # the timed steps are issued by the calling thread (below)
                t0 = time.perf_counter()
                issue = 0.0
                for _ in range(steps):
                    a = time.perf_counter()
                    stats[r] = ex.step()
                    issue += time.perf_counter() - a
                host_us[r] = issue / max(steps, 1) * 1e6
                start.wait()
                if sync_debug and gpu:
                    if r == 0:
                        torch.cuda.set_sync_debug_mode(0)
                    # (process-wide mode: no rank synchronises before rank 0 has switched it off —
                    # rank 2's stream synchronize once raced ahead of it)
                    start.wait()
                if gpu:
                    streams[r].synchronize()
                ms[r] = (time.perf_counter() - t0) / max(steps, 1) * 1e3
        except BaseException as e:  # noqa: BLE001 — reported below, with the rank
            # a step that failed after one of this rank's device-transport waits gave up failed
            # BECAUSE of it (it computed on data that never arrived): report the transport error
            code = 0
            if transport == "device" and not isinstance(e, exm.TransportError):
                try:
                    code = exs[r].transport_errors()
                except Exception:  # noqa: BLE001
                    code = 0
            if code:
                te = exm.TransportError(exs[r]._transport_msg(code))
                te.__cause__ = e
                e = te
            errors.append((r, e))
            start.abort()
            if hasattr(dw, "abort"):  # host transport: the peers' pending waits give up now
                dw.abort()
            if sync_debug and gpu:
                torch.cuda.set_sync_debug_mode(0)

    threads = [threading.Thread(target=drive, args=(r,), daemon=True) for r in range(world)]
    saved = exm.RUNNER_CPU
    exm.RUNNER_CPU = cpu_runner or saved
    try:
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout_s * 2)
    finally:
        exm.RUNNER_CPU = saved
    if any(t.is_alive() for t in threads):
        raise RuntimeError("loopback harness: a rank thread did not finish (hung transfer?)")
    if single_issue and not errors:
        import time

        if not all(ex._graph_exec is not None for ex in exs):
            raise RuntimeError("single_issue needs every rank's step captured as one hipGraph")
        t0 = time.perf_counter()
        for _ in range(steps):
            for r, ex in enumerate(exs):  # (a captured step launches on its rank's own stream)
                stats[r] = ex.step()
        issue = time.perf_counter() - t0
        for r in range(world):
            streams[r].synchronize()
        wall = time.perf_counter() - t0
        host_us = [issue / max(steps * world, 1) * 1e6] * world
        ms = [wall / max(steps, 1) * 1e3] * world
    if gpu:
        torch.cuda.synchronize(device)
    real = [(r, e) for r, e in errors if not isinstance(e, threading.BrokenBarrierError)]
    real.sort(key=lambda re_: not isinstance(re_[1], exm.TransportError))  # the root cause first
    if real or errors:
        r, e = (real or errors)[0]
        raise RuntimeError(f"loopback harness: rank {r} failed: {e!r}") from e
    widened = [[] for _ in range(world)]
    over = [ex.ep_overflow() for ex in exs]
    # an expert-parallel capacity edge overflowed (its routing sent more rows than it holds):
    # every rank widens the groups IT saw overflow — both ranks of a group see the same counts —
    # re-captures, and the whole job runs the step again. A layer's routing depends on the
    # layers before it, so a corrected step can overflow a later layer: repeat until none does
    # (at most once per capacity group)
    rounds = 0
    while ep_exact and any(over):
        rounds += 1
        if rounds > 1 + max(len(ex._ep_groups) for ex in exs):
            raise RuntimeError("loopback harness: expert capacity overflow persists after widening")

        def again(r, _over=over):
            if gpu:
                torch.cuda.set_device(device)
            with (torch.cuda.stream(streams[r]) if gpu else _Null()):
                exs[r].widen_ep(_over[r])
                exs[r].step()  # eager: the widened messages
                if capture and gpu:
                    exs[r].capture()
                stats[r] = exs[r].step()

        _on_ranks(world, again, timeout_s, "re-running a step with widened expert edges")
        if gpu:
            torch.cuda.synchronize(device)
        for r in range(world):
            widened[r] += over[r]
        over = [ex.ep_overflow() for ex in exs]
    hub = getattr(groups[0], "hub", None)
    issue = [ex.issue_mode or ("graph" if ex._graph is not None else None) for ex in exs]
    return LoopbackRun(exs, stats, hub, issue, ms, host_us=host_us, warmup_errors=warm_err,
                       ep_widened=[list(w) for w in widened])


def _on_ranks(world: int, fn, timeout_s: float, what: str) -> None:
    """Run fn(rank) on one thread per rank (their p2p ops pair up) and re-raise a rank's error."""
    errors = []

    def wrap(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errors.append((r, e))

    threads = [threading.Thread(target=wrap, args=(r,), daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout_s * 2)
    if any(t.is_alive() for t in threads):
        raise RuntimeError(f"loopback harness: a rank thread did not finish {what}")
    if errors:
        r, e = errors[0]
        raise RuntimeError(f"loopback harness: rank {r} failed {what}: {e!r}") from e


_RAW_STREAMS: dict = {}


def _rank_streams(device, world: int):
    """Streams for the device transport's ranks: created once per process with hipStreamCreate,
    consecutively — so each sits on a hardware queue of its own (GPU_MAX_HW_QUEUES of them),
    unlike torch's pooled streams, which share queues round-robin (measured:
    benchmarks/hwq_probe.py) — and reused by every later run. A rank's spinning wait must never
    queue another rank's kernels behind it."""
    from .. import ops

    have = _RAW_STREAMS.setdefault(str(device), [])
    while len(have) < world:
        have.append(torch.cuda.ExternalStream(ops.ext().stream_create(), device=device))
    return have[:world]


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
