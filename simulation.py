#!/usr/bin/env python3
"""Reference-compatible evaluation entry point (reference: simulation.py:566-590).

    python simulation.py [--runs 3] [--seed 0] [--out evaluation_results] [--engine native|python]
                         [--schedulers DFS,Greedy,Critical,MRU_spec,EFT,Greedy_chain,MRU_paper]

Sweeps 6 DAG families x {2,4,8} nodes x {100,90,80}% memory x runs x 4 policies and writes
evaluation_results/raw_results.csv (the reference's 14 columns, extra columns appended)
and evaluation_results/scheduler_performance.png, then prints the summary tables.

    python simulation.py --execute [--model gpt2] [--steps 10]      # 1 GPU
    torchrun --nproc-per-node N --master-addr 127.0.0.1 simulation.py --execute   # N GPUs

EXECUTES instead of simulating: every policy x regime places the model's DAG on the job's
GPUs (the reference's node splits and memory formula) and runs it with the native executor;
rows carry the measured ``wall_makespan_ms`` next to the reference columns.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_llm_scheduler_amd.eval.simulation import (DAGGenerator, ImprovedSchedulerEvaluator,  # noqa: E402,F401
                                                           TestResult, main as _main)
from schedulers import *  # noqa: E402,F401,F403


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="evaluation_results")
    ap.add_argument("--engine", choices=["native", "python"], default=None)
    ap.add_argument("--schedulers", default=None,
                    help="comma-separated policy names (default DFS,Greedy,Critical,MRU_spec; also EFT, Greedy_chain, "
                         "MRU_paper)")
    ap.add_argument("--execute", action="store_true", help="run the placed model DAG on this job's devices")
    ap.add_argument("--model", default="gpt2", help="--execute: model DAG (gpt2, gpt2-medium, llama3-8b, ...)")
    ap.add_argument("--steps", type=int, default=10, help="--execute: timed steps per configuration")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--cost-model", default="reference", choices=["reference", "bytes"])
    ap.add_argument("--regimes", default="1.0,0.9,0.8")
    ap.add_argument("--nodes", default="equal", choices=["equal", "reference", "laptops"],
                    help="--execute: memory split over the devices (BASELINE.md 2.3 equal nodes, the sweep's "
                         "heterogeneous split, or test_gpt2.py's 4 laptops)")
    a = ap.parse_args(argv)
    if a.execute:
        return _execute_main(a)
    return _main(num_runs=a.runs, seed=a.seed, out_dir=a.out, engine=a.engine,
                 schedulers=a.schedulers.split(",") if a.schedulers else None)


def _execute_main(a):
    import torch
    import torch.distributed as dist

    from distributed_llm_scheduler_amd.eval import execute

    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpu = torch.cuda.is_available()
    dev = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}") if gpu else None
    if gpu:
        torch.cuda.set_device(dev)
    if world > 1:
        from distributed_llm_scheduler_amd.parallel.comm import init_world

        init_world(int(os.environ.get("RANK", "0")), world, dev)
    try:
        return execute.main(a.model, a.schedulers.split(",") if a.schedulers else None,
                            tuple(float(x) for x in a.regimes.split(",")), a.steps, a.warmup, a.seq,
                            cost_model=a.cost_model, seed=a.seed, out_dir=a.out, nodes=a.nodes)
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
