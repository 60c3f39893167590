"""distributed_llm_scheduler_amd — MI355X-native memory-constrained DAG scheduler + executor.

Layers (see README.md):
  core/      Task/Node data model, the four reference policies (+ XGMI-EFT) on a C++ core
  models/    DAG builders: synthetic families, GPT-2 small/medium, Llama-3-8B, Mixtral-8x7B
  ops/       hand-written HIP/CDNA4 kernels (MFMA GEMM, flash attention, norms, ...)
  parallel/  the executor: per-GPU programs, RCCL p2p edges over xGMI, HBM arena, param cache
  eval/      simulation-compatible evaluation harness (raw_results.csv, 2x2 figure)
  viz/       DAG plots and Gantt charts (planned and measured)
  utils/     tracing (Chrome trace, roctx), config, serialization
"""
from .core import (ALL_SCHEDULERS, SCHEDULERS, BaseScheduler, CriticalPathScheduler, DFSScheduler, EFTScheduler,
                   GreedyChainScheduler, GreedyScheduler, MRUPaperScheduler, MRUScheduler, Node, OpSpec, Task,
                   get_scheduler)

__version__ = "0.1.0"

__all__ = [
    "Task", "Node", "OpSpec", "BaseScheduler", "DFSScheduler", "GreedyScheduler", "CriticalPathScheduler",
    "MRUScheduler", "EFTScheduler", "GreedyChainScheduler", "MRUPaperScheduler", "SCHEDULERS", "ALL_SCHEDULERS", "get_scheduler",
]
