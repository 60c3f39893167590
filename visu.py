#!/usr/bin/env python3
"""Reference-compatible visualisation entry point (reference: visu.py:250-349).

    python visu.py                 # interactive menu (as the reference)
    python visu.py --all [--out d] # batch: write every demo figure to PNG files

Figures: DAG (simple/detailed), the reference's back-to-back Gantt, a dependency-aware
Gantt, and — from an executor run — a measured per-GPU Gantt (see bench.py --profile).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_llm_scheduler_amd.core import MRUScheduler, Node  # noqa: E402
from distributed_llm_scheduler_amd.models.synthetic import (create_mini_llm_dag, create_random_dag,  # noqa: E402
                                                            create_simple_dag)
from distributed_llm_scheduler_amd.viz.plots import (visualize_dag_detailed, visualize_dag_simple,  # noqa: E402
                                                     visualize_schedule_simple)


def test_all_visualizations(out="visu_out", show=False):
    os.makedirs(out, exist_ok=True)
    p = lambda n: os.path.join(out, n)  # noqa: E731
    tasks = create_simple_dag()
    visualize_dag_simple(tasks, "Simple 4-Task DAG", p("simple_dag.png"), show)
    visualize_dag_detailed(tasks, "Simple 4-Task DAG (Detailed)", p("simple_dag_detailed.png"), show)
    llm = create_mini_llm_dag(3)
    visualize_dag_simple(llm, "Mini LLM DAG (3 layers)", p("mini_llm_dag.png"), show)
    visualize_dag_detailed(llm, "Mini LLM DAG (3 layers) - Detailed", p("mini_llm_dag_detailed.png"), show)
    rnd = create_random_dag(15)
    visualize_dag_simple(rnd, "Random DAG (15 tasks)", p("random_dag.png"), show)
    visualize_dag_detailed(rnd, "Random DAG (15 tasks) - Detailed", p("random_dag_detailed.png"), show)
    nodes = [Node("node_0", 5.0, 1.2), Node("node_1", 4.0, 1.0), Node("node_2", 3.0, 0.8)]
    manual = {"node_0": ["t1", "t4"], "node_1": ["t2"], "node_2": ["t3"]}
    visualize_schedule_simple(manual, tasks, nodes, p("gantt_reference_layout.png"), show)
    visualize_schedule_simple(manual, tasks, nodes, p("gantt_with_dependencies.png"), show, respect_deps=True)
    s = MRUScheduler([n.fresh() for n in nodes])
    for t in llm:
        s.add_task(t.clone())
    visualize_schedule_simple(s.schedule(), llm, nodes, p("gantt_mru_mini_llm.png"), show, respect_deps=True)
    visualize_dag_detailed(create_mini_llm_dag(6), "Larger LLM DAG (6 layers)", p("larger_llm_dag.png"), show)
    print(f"wrote figures to {out}/")


def interactive_test():
    while True:
        print("\n" + "=" * 50 + "\nDAG Visualization Tester\n" + "=" * 50)
        print("1. Simple 4-task DAG\n2. Mini LLM DAG (choose layers)\n3. Random DAG (choose size)")
        print("4. Test schedule visualization\n5. Run all tests\n0. Exit")
        c = input("\nEnter your choice: ").strip()
        if c == "0":
            break
        if c == "1":
            t = create_simple_dag()
            visualize_dag_simple(t, "Simple 4-Task DAG", show=True)
            visualize_dag_detailed(t, "Simple 4-Task DAG (Detailed)", show=True)
        elif c == "2":
            n = min(max(int(input("Number of layers (1-10): ")), 1), 10)
            t = create_mini_llm_dag(n)
            visualize_dag_simple(t, f"Mini LLM DAG ({n} layers)", show=True)
            visualize_dag_detailed(t, f"Mini LLM DAG ({n} layers) - Detailed", show=True)
        elif c == "3":
            n = min(max(int(input("Number of tasks (5-50): ")), 5), 50)
            t = create_random_dag(n)
            visualize_dag_simple(t, f"Random DAG ({n} tasks)", show=True)
            visualize_dag_detailed(t, f"Random DAG ({n} tasks) - Detailed", show=True)
        elif c == "4":
            nodes = [Node("GPU_0", 5.0, 1.5), Node("CPU_1", 8.0, 1.0)]
            visualize_schedule_simple({"GPU_0": ["t1", "t3"], "CPU_1": ["t2", "t4"]}, create_simple_dag(), nodes,
                                      show=True)
        elif c == "5":
            test_all_visualizations(show=False)
        else:
            print("Invalid choice!")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--out", default="visu_out")
    a = ap.parse_args()
    if a.all:
        test_all_visualizations(a.out)
    else:
        interactive_test()
