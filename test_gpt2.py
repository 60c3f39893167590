#!/usr/bin/env python3
"""Reference-compatible real-model workflow (reference: test_gpt2.py:246-307).

    python test_gpt2.py [--model gpt2|gpt2-medium] [--out gpt2_dag.pkl]

Builds the GPT-2 operator DAG from local presets (no Hub download), prints the analysis,
saves it (pickle of Task objects, like the reference, plus a JSON export of the DAG IR),
then places it with MRU_spec on four 8/8/6/6 GB "laptops" (reference: 99/99 completed,
24/28/22/25 tasks per node).
"""
import argparse
import json
import os
import pickle
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_llm_scheduler_amd.core import MRUScheduler, Node, Task  # noqa: E402,F401
from distributed_llm_scheduler_amd.models.tracer import LLMDAGExtractor  # noqa: E402
from distributed_llm_scheduler_amd.utils.serialization import save_dag_json  # noqa: E402

LAPTOPS = [("laptop_0", 8.0, 1.0), ("laptop_1", 8.0, 1.2), ("laptop_2", 6.0, 0.8), ("laptop_3", 6.0, 0.9)]


def test_extraction(model="gpt2", out="gpt2_dag.pkl"):
    ex = LLMDAGExtractor(model)
    print(f"Extracting DAG from {model} (local preset)...")
    tasks = ex.extract_gpt2_dag()
    print(f"\nExtracted {len(tasks)} tasks\n\nFirst 5 tasks:")
    for t in tasks[:5]:
        print(f"  {t.id}: mem={t.memory_required:.3f}GB, compute={t.compute_time:.3f}s, deps={t.dependencies}")
    print("\n")
    ex.analyze_dag(tasks)
    if out:
        with open(out, "wb") as f:
            pickle.dump(tasks, f)
        save_dag_json(tasks, os.path.splitext(out)[0] + ".json")
        print(f"\nDAG saved to {out}")
    return tasks


def test_with_your_scheduler(tasks):
    nodes = [Node(i, m, s) for i, m, s in LAPTOPS]
    print("\nTesting MRU Scheduler on real GPT-2 DAG...")
    s = MRUScheduler(nodes)
    for t in tasks:
        s.add_task(t.clone())  # keep the caller's tasks pristine (reference mutates them)
    placed = s.schedule()
    print("MRU Results:")
    print(f"  Completed: {len(s.completed_tasks)}/{len(tasks)}")
    print(f"  Failed: {len(s.failed_tasks)}")
    for nid, tids in placed.items():
        print(f"  {nid}: {len(tids)} tasks")
    return s, placed


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--out", default="gpt2_dag.pkl")
    a = ap.parse_args()
    test_with_your_scheduler(test_extraction(a.model, a.out))
