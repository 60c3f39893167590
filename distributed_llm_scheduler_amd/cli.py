"""Command-line interface: ``python -m distributed_llm_scheduler_amd <command> ...``

Commands (defaults reproduce the reference's settings where one exists, SURVEY §5 "Config"):

  plan      build a model DAG, place it with a policy, lower to per-GPU programs; print the
            placement statistics, optionally save the plan (``--save``) for ``run --resume``
  run       execute a plan on this machine: one process per GPU under torchrun
            (RANK/WORLD_SIZE from the environment), or one CPU/GPU process; prints the
            measured step makespan; ``--trace`` writes a Chrome trace, ``--gantt`` a PNG;
            ``--loopback N`` runs an N-rank plan in one process (``--transport hub|device``).
            A device-transport wait that timed out makes the run invalid: exit code 3
  simulate  the reference evaluation sweep (raw_results.csv + 2x2 figure); --execute runs each
            policy's placement of a model DAG on the devices (measured makespan column)
  extract   the reference GPT-2 DAG (test_gpt2.py semantics) to JSON (test_gpt2.py also pickles it)
  elastic   run with device-loss injection: a worker dies, the DAG is re-planned onto the
            surviving devices and the step is re-executed
  models    list the model presets

Common options: --model, --devices (ignored under torchrun: WORLD_SIZE wins), --scheduler,
--hbm-cap-gb, --cost-model {bytes,reference}, --seq, --batch, --replicas, --placement,
--tp, --sp, --seed, --dtype (bf16 only: the kernels compute in bf16 with fp32 accumulation).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List, Optional


def _common(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--devices", type=int, default=1, help="number of GPUs (overridden by WORLD_SIZE)")
    ap.add_argument("--scheduler", default="EFT",
                    help="DFS | Greedy | Critical | MRU_spec | EFT | Greedy_chain | MRU_paper")
    ap.add_argument("--hbm-cap-gb", type=float, default=288.0, help="per-GPU parameter budget (GB)")
    ap.add_argument("--cost-model", choices=["bytes", "reference"], default="bytes",
                    help="bytes: real tensor sizes; reference: 0.5 GB per parameter, constant compute times")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--replicas", type=int, default=1, help="independent request DAGs (data parallelism)")
    ap.add_argument("--placement", default="scheduler",
                    choices=["scheduler", "replica", "pipeline", "tensor", "sequence"])
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel shards per layer (DAG transform)")
    ap.add_argument("--sp", type=int, default=1, help="sequence chunks per request (context-parallel DAG transform)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16"])
    ap.add_argument("--no-fuse", action="store_true")


def _plan(a, world: int, resume: Optional[str] = None):
    from .parallel import runtime

    return runtime.plan(a.model, world=world, scheduler=a.scheduler, cap_gb=a.hbm_cap_gb, replicas=a.replicas,
                        batch=a.batch, seq=a.seq, cost_model=a.cost_model, fuse=not a.no_fuse,
                        placement=a.placement, tp=a.tp, resume=resume, sp=a.sp)


def cmd_plan(a) -> int:
    from .parallel import runtime

    t0 = time.time()
    p = _plan(a, a.devices)
    out = {"model": a.model, "scheduler": p.scheduler_name, "world": p.world, "plan_ms": round((time.time() - t0) * 1e3, 2)}
    out.update(p.stats)
    print(json.dumps(out))
    if a.save:
        runtime.save_plan(p, a.save)
        print(f"saved plan to {a.save}", file=sys.stderr)
    return 0


def _transport_failure(e: BaseException) -> Optional[str]:
    """The TransportError message in ``e`` or its cause chain (a rank thread's error is re-raised
    by the single-GPU harness as the cause of its RuntimeError), else None."""
    from .parallel.executor import TransportError

    while e is not None:
        if isinstance(e, TransportError):
            return str(e)
        e = e.__cause__
    return None


def cmd_run_loopback(a) -> int:
    """``run --loopback N``: the N-rank plan in THIS process on one device (the single-GPU
    multi-rank harness, parallel/loopback.py): every rank its own executor and thread, edges over
    the loopback hub (``--transport hub``, RCCL's p2p semantics) or moved by kernels (``--transport
    device``, parallel/devp2p.py; on the CPU the same protocol with host waits). A device-transport
    wait that gave up makes the run INVALID: the JSON line says so and the exit code is 3."""
    import torch

    from .parallel.loopback import run_loopback

    gpu = a.device != "cpu" and torch.cuda.is_available()
    dev = torch.device("cuda:0") if gpu else torch.device("cpu")
    p = _plan(a, a.loopback, resume=a.resume)
    out = {"model": a.model, "world": a.loopback, "scheduler": p.scheduler_name, "harness": "loopback",
           "transport": a.transport, "tasks_completed": p.stats["tasks_completed"],
           "tasks_total": p.stats["tasks_total"], "device": str(dev)}
    try:
        from .parallel.devp2p import TIMEOUT_S

        run = run_loopback(p, dev, steps=a.steps, warmup=a.warmup, capture=gpu and not a.no_graph,
                           transport=a.transport, delay_us=0.0, poison=False, p2p_timeout_s=TIMEOUT_S)
        errs = [ex.transport_errors() for ex in run.executors]
        for ex in run.executors:
            ex.check_transport()
    except Exception as e:  # noqa: BLE001
        msg = _transport_failure(e)
        if msg is None:
            raise
        print(json.dumps({**out, "valid": False, "error": msg}))
        print(f"run: INVALID — {msg}", file=sys.stderr)
        return 3
    print(json.dumps({**out, "ms_per_step": round(max(run.step_ms), 4), "p2p_errors": errs, "valid": True}))
    return 0


def cmd_run(a) -> int:
    import torch
    import torch.distributed as dist

    from .parallel import runtime

    if a.loopback:
        return cmd_run_loopback(a)
    world = int(os.environ.get("WORLD_SIZE", a.devices if a.device == "cpu" else 1))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = a.device != "cpu" and torch.cuda.is_available()
    dev = torch.device(f"cuda:{local}") if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    pg = None
    if world > 1:
        if "MASTER_ADDR" not in os.environ:
            raise SystemExit("world > 1 needs torchrun (or MASTER_ADDR/MASTER_PORT/RANK/WORLD_SIZE)")
        from .parallel.comm import init_world

        init_world(rank, world, dev if gpu else None)
        pg = dist.group.WORLD
    p = _plan(a, world, resume=a.resume)
    store = runtime.make_store(p, seed=a.seed, device_init=gpu and a.init == "device" and runtime.device_init_ok(p, rank))
    if gpu and pg is not None:  # DLS_P2P=device: cross-GPU edges moved by kernels (parallel/devp2p.py)
        pg = runtime.p2p_group(p, rank, dev, pg)
    ex = runtime.make_executor(p, rank, dev, store, pg=pg, use_graph=gpu and not a.no_graph, trace=a.roctx)

    def sync():
        if gpu:
            torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    failed: Optional[str] = None  # a device-transport wait gave up on this rank (TransportError)
    try:
        for _ in range(a.warmup):
            ex.step()
    except Exception as e:  # noqa: BLE001
        failed = _transport_failure(e)
        if failed is None:
            raise
    sync()
    while failed is None and runtime.ep_widen_on_overflow(ex, dist.group.WORLD if world > 1 else None):
        ex.step()  # expert capacity edges that overflowed: widened, the step runs again
    sync()
    if gpu and not a.no_graph and failed is None:
        ex.capture()
    sync()
    ex.reset_transport_errors()  # a cold first step may outlast a peer's wait (warm-up only)
    t0 = time.perf_counter()
    try:
        for _ in range(a.steps if failed is None else 0):
            ex.step()
    except Exception as e:  # noqa: BLE001
        failed = _transport_failure(e)
        if failed is None:
            raise
    sync()
    ms = (time.perf_counter() - t0) / max(a.steps, 1) * 1e3
    err = ex.transport_errors()
    if err and failed is None:
        failed = ex._transport_msg(err)
    if failed:
        print(f"run: rank {rank}: INVALID — {failed}", file=sys.stderr)
    t = torch.tensor([ms, 1.0 if failed else 0.0], dtype=torch.float64, device=dev if (gpu and world > 1) else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    invalid = bool(t[1].item())
    events = None
    if (a.trace or a.gantt) and not invalid:
        st = ex.step(profile=True)
        events = [None] * world
        if world > 1:
            dist.all_gather_object(events, st.events)
        else:
            events = [st.events]
    if rank == 0:
        print(json.dumps({"model": a.model, "world": world, "scheduler": p.scheduler_name,
                          "tasks_completed": p.stats["tasks_completed"], "tasks_total": p.stats["tasks_total"],
                          "ms_per_step": round(float(t[0].item()), 4), "device": str(dev),
                          "p2p": getattr(ex.comm, "kind", None), "valid": not invalid}))
        if events is not None:
            from .utils.tracing import chrome_trace, kernel_timeline

            if a.trace:
                chrome_trace(dict(enumerate(events)), a.trace, meta={"model": a.model, "world": world})
            if a.gantt:
                from .viz.plots import measured_gantt

                measured_gantt({r: kernel_timeline(e) for r, e in enumerate(events)}, path=a.gantt)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 3 if invalid else 0


def cmd_simulate(a) -> int:
    if a.execute:  # same policies and regimes, the model DAG RUN on this job's devices
        import torch
        import torch.distributed as dist

        from .eval import execute

        world = int(os.environ.get("WORLD_SIZE", "1"))
        gpu = torch.cuda.is_available()
        dev = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}") if gpu else None
        if gpu:
            torch.cuda.set_device(dev)
        if world > 1:
            from .parallel.comm import init_world

            init_world(int(os.environ.get("RANK", "0")), world, dev)
        try:
            execute.main(a.model, a.schedulers.split(",") if a.schedulers else None,
                         tuple(float(x) for x in a.regimes.split(",")), a.steps, a.warmup, a.seq,
                         cost_model=a.cost_model, seed=a.seed, out_dir=a.out, nodes=a.nodes)
        finally:
            if world > 1:
                dist.destroy_process_group()
        return 0
    from .eval.simulation import main as sim_main

    sim_main(num_runs=a.runs, seed=a.seed, out_dir=a.out, engine=a.engine,
             schedulers=a.schedulers.split(",") if a.schedulers else None)
    return 0


def cmd_extract(a) -> int:
    from .models.tracer import LLMDAGExtractor
    from .utils.serialization import save_dag_json

    if not a.model.startswith("gpt2"):
        raise SystemExit("extract supports the GPT-2 family (reference test_gpt2.py semantics)")
    ex = LLMDAGExtractor(a.model)
    tasks = ex.extract_gpt2_dag(batch=a.batch, seq=a.seq, cost_model=a.cost_model)
    ex.analyze_dag(tasks)
    save_dag_json(tasks, a.out)
    print(f"wrote {len(tasks)} tasks to {a.out}")
    return 0


def cmd_elastic(a) -> int:
    from .parallel.elastic import run_elastic

    out = run_elastic(world=a.devices, steps=a.steps, fail_rank=a.fail_rank, fail_step=a.fail_step,
                      device=a.device, model=a.model, scheduler=a.scheduler, cap_gb=a.hbm_cap_gb,
                      replicas=a.replicas, batch=a.batch, seq=a.seq, cost_model=a.cost_model, placement=a.placement,
                      tp=a.tp, sp=a.sp)
    print(json.dumps(out))
    return 0


def cmd_models(a) -> int:
    from .models.config import PRESETS

    for name, c in sorted(PRESETS.items()):
        print(f"{name:14s} family={c.family:8s} layers={c.n_layer:3d} hidden={c.n_embd:5d} heads={c.n_head:3d} "
              f"kv={c.kv_heads:3d} ffn={c.ffn:6d} vocab={c.vocab_size:6d} experts={c.n_experts}")
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m distributed_llm_scheduler_amd",
                                 description="MI355X-native memory-constrained DAG scheduler + executor")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("plan", help="place a model DAG and print statistics")
    _common(p)
    p.add_argument("--save", default=None, help="write the plan (placement checkpoint) as JSON")
    p.set_defaults(fn=cmd_plan)
    r = sub.add_parser("run", help="execute a placed DAG (torchrun for several GPUs)")
    _common(r)
    r.add_argument("--device", default="auto", choices=["auto", "cpu"])
    r.add_argument("--steps", type=int, default=10)
    r.add_argument("--warmup", type=int, default=2)
    r.add_argument("--resume", default=None, help="use a plan saved by `plan --save` instead of re-scheduling")
    r.add_argument("--init", default="device", choices=["device", "host"])
    r.add_argument("--no-graph", action="store_true")
    r.add_argument("--roctx", action="store_true")
    r.add_argument("--trace", default=None, help="Chrome trace JSON path")
    r.add_argument("--gantt", default=None, help="measured Gantt PNG path")
    r.add_argument("--loopback", type=int, default=0,
                   help="run an N-rank plan in THIS process on one device (single-GPU multi-rank harness)")
    r.add_argument("--transport", default="hub", choices=["hub", "device"],
                   help="--loopback edges: the loopback hub (RCCL semantics) or kernels (device transport)")
    r.set_defaults(fn=cmd_run)
    s = sub.add_parser("simulate", help="reference evaluation sweep")
    s.add_argument("--runs", type=int, default=3)
    s.add_argument("--seed", type=int, default=0)
    s.add_argument("--out", default="evaluation_results")
    s.add_argument("--engine", choices=["native", "python"], default=None)
    s.add_argument("--schedulers", default=None)
    s.add_argument("--execute", action="store_true",
                   help="run each policy's placement of --model on this job's devices (measured makespan column)")
    s.add_argument("--model", default="gpt2")
    s.add_argument("--steps", type=int, default=10)
    s.add_argument("--warmup", type=int, default=3)
    s.add_argument("--seq", type=int, default=512)
    s.add_argument("--cost-model", choices=["bytes", "reference"], default="reference")
    s.add_argument("--regimes", default="1.0,0.9,0.8")
    s.add_argument("--nodes", choices=["equal", "reference", "laptops"], default="equal")
    s.set_defaults(fn=cmd_simulate)
    e = sub.add_parser("extract", help="reference GPT-2 DAG to JSON")
    e.add_argument("--model", default="gpt2")
    e.add_argument("--out", default="gpt2_dag.json")
    e.add_argument("--batch", type=int, default=1)
    e.add_argument("--seq", type=int, default=512)
    e.add_argument("--cost-model", choices=["bytes", "reference"], default="reference")
    e.set_defaults(fn=cmd_extract)
    el = sub.add_parser("elastic", help="run with device-loss injection and re-planning (one process per device)")
    _common(el)
    el.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    el.add_argument("--steps", type=int, default=2)
    el.add_argument("--fail-rank", type=int, default=None)
    el.add_argument("--fail-step", type=int, default=1)
    el.set_defaults(fn=cmd_elastic)
    m = sub.add_parser("models", help="list model presets")
    m.set_defaults(fn=cmd_models)
    a = ap.parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
