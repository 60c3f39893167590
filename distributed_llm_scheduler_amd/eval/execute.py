"""Executed evaluation: the reference sweep's policies x memory regimes on a MODEL DAG,
placed by each policy and then RUN by the native executor on the GPUs of this job.

The reference only simulates (``simulation.py:216-278`` replays compute constants and
ignores dependencies); BASELINE.md §3 asks for the tasks completed under the
same DAG / memory budget / regime together with a measured wall-clock makespan. One row
per (policy, regime), in the reference's ``raw_results.csv`` format:

* the reference columns come from the same formulas as the simulated sweep
  (:class:`ImprovedSchedulerEvaluator`): heterogeneous node construction
  (``simulation.py:161-192``: 60/40 at 2 nodes, 35/25/25/15 at 4, equal otherwise), the
  "100 % memory" total (``simulation.py:194-214``), the dependency-free makespan and load
  balance of the placement;
* appended columns: ``wall_makespan_ms`` — the measured step time of the placed DAG (max
  over ranks: every kernel, parameter refill the policy's evict/reload trace causes, and
  RCCL p2p transfer), ``hbm_peak_gb`` (the largest rank's activation + parameter +
  workspace arenas), ``bytes_moved_p2p`` and ``param_fill_bytes`` per steady-state step
  (all ranks), ``device``.

Tasks the policy failed (or orphaned) are not executed — exactly the reference's
completion semantics. World size = the torch.distributed job (``torchrun`` for >1 GPU,
RCCL on GPUs, gloo on CPU); every rank runs the same configurations in the same order and
rank 0 writes the CSV.
"""
from __future__ import annotations

import random
import time
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..core.schedulers import ALL_SCHEDULERS, SCHEDULERS
from ..models import registry
from .simulation import ImprovedSchedulerEvaluator, TestResult

DAG_TYPE = {"gpt2": "LLM-GPT2", "gpt2-medium": "LLM-GPT2-medium", "llama3-8b": "LLM-Llama3-8B",
            "mixtral-8x7b": "LLM-Mixtral-8x7B"}


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _reduce(x: float, op, device) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return float(t.item())


def run_executed(model: str = "gpt2", schedulers: Optional[Sequence[str]] = None,
                 regimes: Sequence[float] = (1.0, 0.9, 0.8), steps: int = 10, warmup: int = 3, seq: int = 512,
                 batch: int = 1, cost_model: str = "reference", seed: int = 0, device=None,
                 use_graph: bool = True, verbose: bool = True, nodes: str = "equal") -> List[TestResult]:
    """Plan + execute ``model``'s DAG for every (policy, regime) on this job's devices.

    ``nodes``: how the regime's memory is split over the devices —
    ``"equal"`` (BASELINE.md §2.3's GPT-2 grid: N equal nodes at speed 1.0),
    ``"reference"`` (the sweep's construction, simulation.py:161-192) or ``"laptops"``
    (test_gpt2.py:278-283: 8/8/6/6 GB at speeds 1.0/1.2/0.8/0.9 whatever the regime; 4 devices)."""
    from ..parallel import runtime

    rank, world = _world()
    if device is None:
        device = torch.device(f"cuda:{torch.cuda.current_device()}") if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    gpu = device.type == "cuda"
    pg = dist.group.WORLD if world > 1 else None
    names = list(schedulers) if schedulers else list(SCHEDULERS)
    ev = ImprovedSchedulerEvaluator({n: ALL_SCHEDULERS[n] for n in names}, seed=seed, verbose=False)
    tasks, groups, _ = registry.build(model, batch=batch, seq=seq, cost_model=cost_model)
    if cost_model == "reference":
        total = ev.calculate_total_memory_needed(tasks)
    else:  # same formula with each parameter group's real size (GB)
        from ..models.params import group_layout
        gb = {pid: group_layout(g)[0] / 1e9 for pid, g in groups.items()}
        total = max(t.memory_required + sum(gb[p] for p in t.params_needed) for t in tasks) + sum(gb.values())
    dev_name = torch.cuda.get_device_name(device) if gpu else "cpu"
    rows: List[TestResult] = []
    stores = {}  # device_init flag -> ParamStore, shared by every configuration (same weights)
    for regime in regimes:
        spec = _node_spec(ev, nodes, total, regime, world, seed)
        for name in names:
            t0 = time.perf_counter()
            p = runtime.plan(model, world=world, scheduler=name, cap_gb=[m for m, _ in spec],
                             node_speeds=[v for _, v in spec], seq=seq, batch=batch,
                             cost_model=cost_model)
            decide = time.perf_counter() - t0
            sched, schedule = p.scheduler, p.schedule
            makespan, st = ev.simulate_execution(sched, schedule)
            util = sum(st["node_utilization"].values()) / len(st["node_utilization"]) if st["node_utilization"] else 0
            loads = sum(1 for e in sched.events if e[1] == "LOAD")
            evicts = sum(1 for e in sched.events if e[1] == "EVICT")
            done, failed = len(sched.completed_tasks), len(sched.failed_tasks)
            wall, hbm, p2p, fills = _execute(p, rank, device, pg, steps, warmup, use_graph, gpu, stores)
            row = TestResult(
                name, DAG_TYPE.get(model, f"LLM-{model}"), regime, len(tasks), done, failed, makespan, util,
                st["param_cache_hits"], st["param_cache_misses"], ev.calculate_load_balance(sched, schedule),
                decide, done / len(tasks) * 100, world, ev.dependency_makespan(sched, schedule),
                len(sched.orphaned_tasks), loads, evicts, getattr(sched, "rounds", 0),
                "native" if getattr(sched, "_native_result", None) is not None else "python", seed, wall,
                hbm, p2p, fills, dev_name)
            rows.append(row)
            if verbose and rank == 0:
                print(f"[execute] {model} x{world} {name:9s} @{regime:.0%}: {done}/{len(tasks)} tasks, "
                      f"{wall:.3f} ms/step measured, {fills / 1e6:.1f} MB refilled/step, "
                      f"{p2p / 1e6:.2f} MB p2p/step, ref makespan {makespan:.3f}", flush=True)
    return rows


def regime_node_spec(model: str, regime: float, world: int, batch: int = 1, seq: int = 512, seed: int = 0):
    """[(memory GB, speed)] per GPU for ONE request DAG of ``model`` spread over ``world`` nodes:
    the reference's memory regime over its total-need formula (simulation.py:194-214, its
    0.5 GB-per-parameter cost model) split as the reference splits it (simulation.py:161-192:
    60/40 at 2 nodes, 35/25/25/15 at 4, equal shares with seeded speeds otherwise)."""
    tasks, _, _ = registry.build(model, batch=batch, seq=seq, cost_model="reference")
    ev = ImprovedSchedulerEvaluator({}, seed=seed, verbose=False)
    total = ev.calculate_total_memory_needed(tasks)
    return _node_spec(ev, "reference" if world > 1 else "equal", total, regime, world, seed)


def _node_spec(ev, mode, total, regime, world, seed):
    """[(memory GB, speed)] per device."""
    if mode == "equal":
        return [(total * regime / world, 1.0)] * world
    if mode == "laptops":
        if world != 4:
            raise ValueError("the laptops configuration has 4 devices")
        return [(8.0, 1.0), (8.0, 1.2), (6.0, 0.8), (6.0, 0.9)]
    if mode == "reference":
        ev.rng = random.Random(seed)  # identical node speeds on every rank and for every policy
        return [(n.total_memory, n.compute_speed) for n in ev.create_nodes_with_memory_regime(total, regime, world)]
    raise ValueError(f"unknown node construction {mode!r}")


def _execute(p, rank, device, pg, steps, warmup, use_graph, gpu, stores=None):
    """(wall ms per step max over ranks, peak HBM GB max over ranks, p2p bytes and
    parameter-fill bytes per steady-state step summed over ranks)."""
    from ..parallel import runtime

    # device RNG init straight into HBM, unless the program re-fills groups in the steady
    # state: then every refill must be a real host->HBM copy
    dev_init = gpu and runtime.device_init_ok(p, rank)
    stores = {} if stores is None else stores
    if dev_init not in stores:
        stores[dev_init] = runtime.make_store(p, device_init=dev_init)
    store = stores[dev_init]
    ex = runtime.make_executor(p, rank, device, store, pg=pg, use_graph=use_graph)
    stats = None
    for _ in range(max(warmup, 2)):
        stats = ex.step()  # the last eager step is a steady-state one (residency warmed)
    _sync(gpu, device, pg)
    if use_graph and ex.capture():
        ex.step()
    _sync(gpu, device, pg)
    t0 = time.perf_counter()
    for _ in range(steps):
        ex.step()
    _sync(gpu, device, pg)
    wall = (time.perf_counter() - t0) / max(steps, 1) * 1e3
    mem = ex.memory_bytes()
    hbm = (mem["activations"] + mem["params"] + mem["workspace"]) / 1e9
    out = (_reduce(wall, dist.ReduceOp.MAX, device if gpu else "cpu"),
           _reduce(hbm, dist.ReduceOp.MAX, device if gpu else "cpu"),
           _reduce(float(stats.bytes_sent), dist.ReduceOp.SUM, device if gpu else "cpu"),
           _reduce(float(stats.bytes_filled), dist.ReduceOp.SUM, device if gpu else "cpu"))
    del ex, store
    if gpu:
        torch.cuda.empty_cache()
    return out


def _sync(gpu, device, pg):
    if gpu:
        torch.cuda.synchronize(device)
    if pg is not None:
        dist.barrier()


def main(model: str = "gpt2", schedulers: Optional[Sequence[str]] = None, regimes=(1.0, 0.9, 0.8),
         steps: int = 10, warmup: int = 3, seq: int = 512, cost_model: str = "reference", seed: int = 0,
         out_dir: str = "evaluation_results", plot: bool = True, nodes: str = "equal"):
    """``python simulation.py --execute``: rows -> ``out_dir/raw_results.csv`` (rank 0)."""
    import os

    rank, world = _world()
    rows = run_executed(model, schedulers, regimes, steps, warmup, seq, cost_model=cost_model, seed=seed,
                        nodes=nodes)
    if rank == 0:
        ev = ImprovedSchedulerEvaluator({}, seed=seed, verbose=False)
        ev.results = rows
        df = ev.analyze_results(out_dir, plot=plot)
        if df is not None:
            cols = ["scheduler_name", "memory_regime", "completed_tasks", "total_tasks", "makespan",
                    "wall_makespan_ms", "param_fill_bytes", "bytes_moved_p2p", "hbm_peak_gb"]
            print("\n=== EXECUTED ON", rows[0].device if rows else "?", f"x{world} ===")
            print(df[cols].to_string(index=False))
        print(f"\nEvaluation complete! Check '{os.path.abspath(out_dir)}' for raw_results.csv.")
    return rows
