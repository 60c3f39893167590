#!/usr/bin/env python3
"""Reference-compatible module: ``from schedulers import *`` gives Task, Node, BaseScheduler
and the four policies (plus the new EFTScheduler), backed by the native C++ core.

``python schedulers.py`` runs the 4-task diamond smoke demo on two devices
(reference: schedulers.py:528-572)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_llm_scheduler_amd.core import (BaseScheduler, CriticalPathScheduler, DFSScheduler,  # noqa: E402,F401
                                                EFTScheduler, GreedyScheduler, MRUScheduler, Node, Task)
from distributed_llm_scheduler_amd.models.synthetic import create_simple_dag  # noqa: E402

__all__ = ["Task", "Node", "BaseScheduler", "DFSScheduler", "GreedyScheduler", "CriticalPathScheduler",
           "MRUScheduler", "EFTScheduler", "test_schedulers"]


def test_schedulers():
    print("Testing Schedulers\n")
    tasks = create_simple_dag()
    devices = [("n1", 3.0), ("n2", 2.5)]
    policies = {"DFS": DFSScheduler, "Greedy": GreedyScheduler, "Critical Path": CriticalPathScheduler,
                "MRU_spec": MRUScheduler, "XGMI-EFT": EFTScheduler}
    for label, cls in policies.items():
        print(f"\n{label}:")
        s = cls([Node(i, m) for i, m in devices])
        for t in tasks:
            s.add_task(copy.deepcopy(t))
        placed = s.schedule()
        print(f"  Completed: {len(s.completed_tasks)}/{len(tasks)}")
        print(f"  Failed: {len(s.failed_tasks)}")
        print(f"  Schedule: {dict(placed)}")


if __name__ == "__main__":
    test_schedulers()
