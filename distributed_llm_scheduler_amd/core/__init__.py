from .task import Node, OpSpec, Task, clone_nodes, clone_tasks
from .schedulers import (ALL_SCHEDULERS, SCHEDULERS, BaseScheduler, CriticalPathScheduler, DFSScheduler,
                         EFTScheduler, GreedyChainScheduler, GreedyScheduler, MRUPaperScheduler, MRUScheduler, bottom_levels, default_engine, get_scheduler,
                         task_depths)

__all__ = [
    "Task", "Node", "OpSpec", "clone_tasks", "clone_nodes", "BaseScheduler", "DFSScheduler", "GreedyScheduler",
    "CriticalPathScheduler", "MRUScheduler", "EFTScheduler", "GreedyChainScheduler", "MRUPaperScheduler", "SCHEDULERS", "ALL_SCHEDULERS", "get_scheduler",
    "default_engine", "task_depths", "bottom_levels",
]
