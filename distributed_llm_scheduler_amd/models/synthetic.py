"""Synthetic DAG families used by the evaluation sweep.

Same shapes, ids, costs and random-number call sequence as the reference generators
(``/root/reference/simulation.py:33-151``, ``visu.py:24-85``), so that seeding Python's
``random`` identically reproduces the reference's DAGs. Every generator also accepts an
explicit ``rng`` (``random.Random``) for reproducible sweeps without global state.
"""
from __future__ import annotations

import random as _random
from typing import List, Optional

from ..core.task import Task


def _rng(rng: Optional[_random.Random]):
    return rng if rng is not None else _random


class DAGGenerator:
    """Reference-compatible generator namespace (``DAGGenerator.generate_*``)."""

    @staticmethod
    def generate_llm_dag(num_layers: int, layer_width: int = 1, attention_heads: int = 8,
                         ffn_multiplier: int = 4) -> List[Task]:
        """embedding → per layer [≤4 parallel head tasks → attention_output → ffn → output] → output.

        ``layer_width`` and ``ffn_multiplier`` are accepted for signature compatibility and,
        as in the reference, do not change the graph (simulation.py:37-88).
        """
        heads = min(attention_heads, 4)
        out = [Task("embedding", 0.5, 0.1, [], {"embedding_weights"})]
        prev = "embedding"
        for layer in range(num_layers):
            head_ids = []
            for h in range(heads):
                tid = f"layer_{layer}_attention_head_{h}"
                out.append(Task(tid, 0.2, 0.05, [prev], {f"layer_{layer}_attention_head_{h}_weights"}))
                head_ids.append(tid)
            out.append(Task(f"layer_{layer}_attention_output", 0.3, 0.05, head_ids,
                            {f"layer_{layer}_attention_output_weights"}))
            out.append(Task(f"layer_{layer}_ffn", 0.5, 0.1, [f"layer_{layer}_attention_output"],
                            {f"layer_{layer}_ffn_weights"}))
            out.append(Task(f"layer_{layer}_output", 0.1, 0.02, [f"layer_{layer}_ffn"], set()))
            prev = f"layer_{layer}_output"
        out.append(Task("output", 0.3, 0.05, [prev], {"output_weights"}))
        return out

    @staticmethod
    def generate_random_dag(num_tasks: int, max_deps: int = 3, rng: Optional[_random.Random] = None) -> List[Task]:
        r = _rng(rng)
        out = []
        for i in range(num_tasks):
            deps: List[str] = []
            if i > 0:
                k = min(r.randint(0, min(max_deps, i)), i)
                if k > 0:
                    deps = r.sample([f"task_{j}" for j in range(i)], k)
            n_params = r.randint(1, 2)
            params = {f"param_{i}_{j}" for j in range(n_params)}
            mem = r.uniform(0.1, 0.5)
            comp = r.uniform(0.05, 0.15)
            out.append(Task(f"task_{i}", mem, comp, deps, params))
        return out

    @staticmethod
    def generate_pipeline_dag(num_stages: int, width: int = 3) -> List[Task]:
        """Stages of ``width`` workers, fully connected stage to stage, one shared parameter
        per stage; a final aggregation task (the only reference workload with sharing)."""
        out = []
        for s in range(num_stages):
            deps = [] if s == 0 else [f"stage_{s - 1}_worker_{i}" for i in range(width)]
            for w in range(width):
                out.append(Task(f"stage_{s}_worker_{w}", 0.3, 0.1, list(deps), {f"stage_{s}_params"}))
        out.append(Task("final_output", 0.2, 0.05, [f"stage_{num_stages - 1}_worker_{i}" for i in range(width)],
                        {"output_params"}))
        return out


# --- visualisation demo DAGs (visu.py:24-85) -----------------------------------------

def create_simple_dag() -> List[Task]:
    """The 4-task diamond t1 → {t2, t3} → t4 used by every smoke demo."""
    return [
        Task("t1", 1.0, 0.1, [], {"p1"}),
        Task("t2", 1.0, 0.1, ["t1"], {"p2"}),
        Task("t3", 1.0, 0.1, ["t1"], {"p3"}),
        Task("t4", 1.0, 0.1, ["t2", "t3"], {"p1", "p2"}),
    ]


def create_mini_llm_dag(num_layers: int = 3) -> List[Task]:
    out = [Task("embedding", 0.5, 0.1, [], {"embedding_weights"})]
    prev = "embedding"
    for i in range(num_layers):
        out.append(Task(f"layer_{i}_attention", 0.3, 0.05, [prev], {f"layer_{i}_attn_weights"}))
        out.append(Task(f"layer_{i}_ffn", 0.5, 0.1, [f"layer_{i}_attention"], {f"layer_{i}_ffn_weights"}))
        out.append(Task(f"layer_{i}_output", 0.1, 0.02, [f"layer_{i}_ffn"], set()))
        prev = f"layer_{i}_output"
    out.append(Task("output", 0.3, 0.05, [prev], {"output_weights"}))
    return out


def create_random_dag(n: int = 10, rng: Optional[_random.Random] = None) -> List[Task]:
    r = _rng(rng)
    out = []
    for i in range(n):
        deps: List[str] = []
        if i > 0:
            k = min(r.randint(0, 2), i)
            if k > 0:
                deps = r.sample([f"task_{j}" for j in range(i)], k)
        mem = r.uniform(0.2, 0.8)
        comp = r.uniform(0.05, 0.2)
        out.append(Task(f"task_{i}", mem, comp, deps, {f"param_{i}"}))
    return out
