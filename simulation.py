#!/usr/bin/env python3
"""Reference-compatible evaluation entry point (reference: simulation.py:566-590).

    python simulation.py [--runs 3] [--seed 0] [--out evaluation_results] [--engine native|python]
                         [--schedulers DFS,Greedy,Critical,MRU_spec,EFT,Greedy_chain,MRU_paper]

Sweeps 6 DAG families x {2,4,8} nodes x {100,90,80}% memory x runs x 4 policies and writes
evaluation_results/raw_results.csv (the reference's 14 columns, extra columns appended)
and evaluation_results/scheduler_performance.png, then prints the summary tables.
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
    a = ap.parse_args(argv)
    return _main(num_runs=a.runs, seed=a.seed, out_dir=a.out, engine=a.engine,
                 schedulers=a.schedulers.split(",") if a.schedulers else None)


if __name__ == "__main__":
    main()
