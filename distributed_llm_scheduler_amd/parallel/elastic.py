"""Elastic execution: device-loss injection and re-planning onto the survivors
(SURVEY §5 "Failure detection / elastic": the reference only knows *scheduling* failure).

:func:`run_elastic` is a small supervisor. It launches one worker process per device (the
same one-process-per-GPU layout as ``torchrun``; ``gloo`` on CPU, ``nccl``=RCCL on GPUs),
each planning deterministically and executing ``steps`` DAG steps. A worker can be told to
die at a given step (``fail_rank`` / ``fail_step``: the process exits abruptly, as a lost
GPU would take its process down). The supervisor notices the dead worker, stops the
others (their peers' p2p operations can no longer complete), re-plans the DAG on the
surviving devices with :func:`runtime.replan` and relaunches — the placement policy, the
per-GPU memory cap and the memory accounting are unchanged, only the device set shrinks.
"""
from __future__ import annotations

import os
import socket
import time
from typing import Dict, List, Optional, Sequence

import torch.multiprocessing as mp

FAIL_EXIT_CODE = 17


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, plan_kw: Dict, steps: int, device: str, fail: Optional[tuple], q,
            devices: Optional[Sequence[int]] = None):
    import torch
    import torch.distributed as dist

    from . import runtime

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    gpu = device == "cuda"
    # rank -> physical GPU: after a loss the survivors are renumbered 0..n-1 but keep their
    # own devices (rank 1 of 3 lost: new ranks 0, 1 run on cuda:0, cuda:2)
    phys = devices[rank] if devices is not None else rank
    dev = torch.device(f"cuda:{phys}") if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    # device_id binds the NCCL (RCCL) communicator to this GPU eagerly, and the barrier runs one
    # collective on the whole group before any step: a rank whose first p2p point posts a
    # batch_isend_irecv group may then never be the one that initialises the communicator
    # (undefined for a batch that is the group's first collective and not every rank's)
    from .comm import init_world

    init_world(rank, world, dev if gpu else None)
    try:
        p = runtime.plan(world=world, **plan_kw)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, dev, store, pg=dist.group.WORLD, use_graph=False)
        for step in range(steps):
            if fail is not None and fail[0] == rank and fail[1] == step:
                os._exit(FAIL_EXIT_CODE)  # simulated device loss: no cleanup, no goodbye
            ex.step()
        if gpu:
            torch.cuda.synchronize(dev)
        res = {"rank": rank, "device": phys, "ok": True, "tasks": sum(1 for r in p.placement.values() if r == rank)}
        head = [t for t in p.placement if t.split("/")[-1] == "output_projection" and p.placement[t] == rank]
        if head:
            res["logits_sum"] = {t: float(ex.output(t).float().sum()) for t in head}
        q.put(res)
    finally:
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def _launch(world: int, plan_kw: Dict, steps: int, device: str, fail: Optional[tuple], timeout: float,
            devices: Optional[Sequence[int]] = None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    devices = list(devices) if devices is not None else list(range(world))
    procs = [ctx.Process(target=_worker, args=(r, world, port, plan_kw, steps, device, fail, q, devices))
             for r in range(world)]
    for pr in procs:
        pr.start()
    deadline = time.time() + timeout
    lost: List[int] = []
    while time.time() < deadline:
        codes = [pr.exitcode for pr in procs]
        lost = [r for r, c in enumerate(codes) if c not in (None, 0)]
        if lost or all(c == 0 for c in codes):
            break
        time.sleep(0.05)
    if lost or any(pr.exitcode is None for pr in procs):
        for pr in procs:  # our own worker handles only
            if pr.exitcode is None:
                pr.terminate()
        for pr in procs:
            pr.join(timeout=10)
        if not lost:
            lost = [r for r, pr in enumerate(procs) if pr.exitcode not in (0,)]
    results = []
    while not q.empty():
        results.append(q.get())
    return lost, sorted(results, key=lambda r: r["rank"])


def run_elastic(world: int, steps: int = 2, fail_rank: Optional[int] = None, fail_step: int = 1,
                device: str = "cpu", timeout: float = 300.0, max_restarts: int = 2,
                devices: Optional[Sequence[int]] = None, **plan_kw) -> Dict:
    """Run ``steps`` DAG steps on ``world`` devices, surviving device loss by re-planning.
    ``plan_kw`` are :func:`runtime.plan` arguments (model, scheduler, cap_gb, replicas, ...);
    ``devices`` the physical GPU of each initial rank (default 0..world-1). Returns the
    attempts (world size, lost ranks, physical devices) and the final per-rank results."""
    from . import runtime

    attempts = []
    fail = (fail_rank, fail_step) if fail_rank is not None else None
    cur = world
    devs = list(devices) if devices is not None else list(range(world))
    if len(devs) != world:
        raise ValueError(f"{len(devs)} devices given for world {world}")
    kw = dict(plan_kw)
    for _ in range(max_restarts + 1):
        lost, results = _launch(cur, kw, steps, device, fail, timeout, devs)
        attempts.append({"world": cur, "lost": lost, "devices": list(devs)})
        if not lost:
            return {"attempts": attempts, "world": cur, "devices": devs, "results": results}
        base = runtime.plan(world=cur, **kw)
        new = runtime.replan(base, lost)
        # the survivors keep their physical devices and (via replan) their node speeds
        devs = [d for r, d in enumerate(devs) if r not in set(lost)]
        cur = new.world
        kw = {k: v for k, v in new.args.items() if k != "world"}
        fail = None  # the injected loss happened once
    raise RuntimeError(f"giving up after {len(attempts)} attempts: {attempts}")
