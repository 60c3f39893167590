"""Model registry: preset name -> (task DAG, parameter groups, config)."""
from __future__ import annotations

from typing import Dict, List, Tuple

from ..core.task import Task
from .config import ModelConfig, get_config
from .params import ParamGroup


def param_groups(cfg: ModelConfig) -> Dict[str, ParamGroup]:
    if cfg.family == "gpt2":
        from .gpt2 import gpt2_param_groups
        return gpt2_param_groups(cfg)
    if cfg.family in ("llama", "mixtral"):
        from .llama import llama_param_groups
        return llama_param_groups(cfg)
    raise KeyError(cfg.family)


def build_dag(cfg: ModelConfig, batch: int = 1, seq: int = 512, cost_model: str = "bytes",
              prefix: str = "") -> List[Task]:
    if cfg.family == "gpt2":
        from .gpt2 import build_gpt2_dag
        return build_gpt2_dag(cfg, batch=batch, seq=seq, cost_model=cost_model, prefix=prefix)
    if cfg.family in ("llama", "mixtral"):
        from .llama import build_llama_dag
        return build_llama_dag(cfg, batch=batch, seq=seq, cost_model=cost_model, prefix=prefix)
    raise KeyError(cfg.family)


def build(model: str, batch: int = 1, seq: int = 512, replicas: int = 1, cost_model: str = "bytes",
          tp: int = 1, sp: int = 1) -> Tuple[List[Task], Dict[str, ParamGroup], ModelConfig]:
    """``replicas`` independent requests (task ids prefixed ``r{k}/``) sharing weights;
    ``tp > 1`` splits every layer into tensor-parallel shards, ``sp > 1`` every token-wise
    node into sequence chunks (models/transforms.py)."""
    cfg = get_config(model)
    tasks: List[Task] = []
    for r in range(replicas):
        tasks.extend(build_dag(cfg, batch, seq, cost_model, prefix=f"r{r}/" if replicas > 1 else ""))
    groups = param_groups(cfg)
    if tp > 1:
        from .transforms import tensor_parallel
        tasks, groups = tensor_parallel(tasks, groups, cfg, tp)
    if sp > 1:
        if tp > 1:
            raise ValueError("combine sequence and tensor parallelism through separate DAGs (not both)")
        from .transforms import sequence_parallel
        tasks, groups = sequence_parallel(tasks, groups, cfg, sp)
    return tasks, groups, cfg
