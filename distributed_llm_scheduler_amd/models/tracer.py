"""DAG extraction from real PyTorch models (reference ``LLMDAGExtractor``, test_gpt2.py:11-243).

* :meth:`LLMDAGExtractor.extract_gpt2_dag` — the hand-written 99-task GPT-2 graph, built
  from local config presets (no Hub download) with real op specs attached.
* :meth:`LLMDAGExtractor.extract_from_traced_model` — a *dataflow* tracer. The reference's
  forward-hook tracer links each op to ``op_{i-1}`` while naming tasks
  ``op_{i}_{name}``, so only one task can ever complete, and it misses functional ops
  such as attention cores and residual adds. Here every torch-level call is
  intercepted with a ``TorchFunctionMode``; tensors are tracked by identity, so each
  task's dependencies are the tasks that produced its input tensors. ``granularity=
  "module"`` groups calls by the innermost leaf module (hooks supply the names),
  ``"op"`` keeps one task per call.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
from torch.overrides import TorchFunctionMode

from ..core.task import Task
from .config import get_config
from .gpt2 import build_gpt2_dag

_SKIP = {"size", "dim", "__get__", "__len__", "numel", "is_contiguous", "stride", "data_ptr", "__format__",
         "__repr__", "__bool__", "__int__", "__float__", "requires_grad_", "get_device", "storage_offset",
         "element_size", "__eq__", "__hash__", "__setstate__", "__reduce_ex__", "_has_compatible_shallow_copy_type"}


class _Recorder(TorchFunctionMode):
    def __init__(self, owner):
        super().__init__()
        self.owner = owner

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        name = getattr(func, "__name__", str(func))
        if name not in _SKIP:
            self.owner._record(name, args, kwargs, out)
        return out


class LLMDAGExtractor:
    def __init__(self, model_name: str = "gpt2"):
        self.model_name = model_name
        self.tasks: List[Task] = []

    # ---- cost estimates (reference formulas, test_gpt2.py:18-43) -----------------
    @staticmethod
    def estimate_memory_gb(module: nn.Module, input_shape) -> float:
        params = sum(p.numel() * 4 for p in module.parameters()) / 1e9
        if hasattr(module, "weight") and isinstance(getattr(module, "weight"), torch.Tensor):
            batch = input_shape[0] if input_shape else 1
            act = np.prod(module.weight.shape) * batch * 4 / 1e9
        else:
            act = 0.1
        return params + act

    @staticmethod
    def estimate_compute_time(module: nn.Module) -> float:
        if isinstance(module, nn.MultiheadAttention):
            return 0.05
        if isinstance(module, nn.Linear):
            return 0.1 if module.out_features > 2048 else 0.03
        return 0.02

    # ---- hand-written GPT-2 graph ------------------------------------------------
    def extract_gpt2_dag(self, batch: int = 1, seq: int = 512, cost_model: str = "reference") -> List[Task]:
        preset = {"gpt2": "gpt2", "gpt2-small": "gpt2", "gpt2-medium": "gpt2-medium"}.get(self.model_name,
                                                                                          self.model_name)
        self.tasks = build_gpt2_dag(get_config(preset), batch=batch, seq=seq, cost_model=cost_model)
        return self.tasks

    # ---- dataflow tracer ----------------------------------------------------------
    def _record(self, name, args, kwargs, out):
        deps = []
        in_bytes = 0

        def visit(x):
            nonlocal in_bytes
            if isinstance(x, torch.Tensor):
                prod = self._producer.get(id(x))
                if prod is not None and prod not in deps:
                    deps.append(prod)
                in_bytes += x.numel() * x.element_size()
            elif isinstance(x, (list, tuple)):
                for y in x:
                    visit(y)

        visit(args)
        visit(list(kwargs.values()))
        outs = out if isinstance(out, (list, tuple)) else [out]
        tensors = [o for o in outs if isinstance(o, torch.Tensor)]
        if not tensors:
            return
        module = self._stack[-1] if self._stack else ""
        flops = 0.0
        if name in ("linear", "matmul", "mm", "bmm", "addmm", "baddbmm", "__matmul__", "conv1d"):
            a = [x for x in (args if isinstance(args, (list, tuple)) else [args]) if isinstance(x, torch.Tensor)]
            if len(a) >= 2:
                k = a[0].shape[-1]
                flops = 2.0 * tensors[0].numel() * k
        key = module if self._granularity == "module" and module else None
        if key is not None and self._ops and self._ops[-1]["key"] == key:
            op = self._ops[-1]
            op["deps"].extend(d for d in deps if d != op["idx"] and d not in op["deps"])
            op["flops"] += flops
        else:
            op = {"idx": len(self._ops), "key": key, "name": name, "module": module, "deps": deps, "flops": flops,
                  "out_bytes": 0}
            self._ops.append(op)
        op["out_bytes"] = sum(t.numel() * t.element_size() for t in tensors)
        for t in tensors:
            self._producer[id(t)] = op["idx"]
            self._keep.append(t)

    def extract_from_traced_model(self, model: nn.Module, sample_input, granularity: str = "module",
                                  param_cost_model: str = "reference") -> List[Task]:
        """Trace one forward pass; return tasks with correct dataflow dependencies."""
        self._producer: Dict[int, int] = {}
        self._ops: List[dict] = []
        self._stack: List[str] = []
        self._keep: List[torch.Tensor] = []
        self._granularity = granularity
        hooks = []
        leaf = {n: m for n, m in model.named_modules() if len(list(m.children())) == 0}

        def enter(n):
            def pre(mod, inp):
                self._stack.append(n)  # returns None: inputs untouched
            return pre

        def leave(mod, inp, out):
            self._stack.pop()  # must return None, or the hook would replace the output

        for n, m in leaf.items():
            hooks.append(m.register_forward_pre_hook(enter(n)))
            hooks.append(m.register_forward_hook(leave))
        try:
            with torch.no_grad(), _Recorder(self):
                if isinstance(sample_input, dict):
                    model(**sample_input)
                else:
                    model(sample_input)
        finally:
            for h in hooks:
                h.remove()
        tasks = []
        ids = []
        for op in self._ops:
            label = (op["key"] or f"{op['module']}.{op['name']}" if op["module"] else op["name"]).replace(".", "_")
            ids.append(f"op_{op['idx']}_{label}")
        for op, tid in zip(self._ops, ids):
            mod = leaf.get(op["module"]) if op["module"] else None
            params = set()
            if mod is not None and list(mod.parameters()):
                params = {f"{op['module']}_params"}
            mem = self.estimate_memory_gb(mod, (1,)) if (mod is not None and param_cost_model == "reference") \
                else op["out_bytes"] / 1e9
            comp = self.estimate_compute_time(mod) if mod is not None else 0.01
            tasks.append(Task(tid, float(mem), comp, [ids[d] for d in op["deps"]], params, None, op["out_bytes"],
                              op["flops"]))
        self.tasks = tasks
        self._keep = []
        return tasks

    # ---- summary --------------------------------------------------------------------
    @staticmethod
    def analyze_dag(tasks: List[Task], param_cost: float = 0.5, verbose: bool = True) -> dict:
        params = set()
        for t in tasks:
            params.update(t.params_needed)
        info = {
            "total_tasks": len(tasks),
            "total_memory_gb": sum(t.memory_required for t in tasks),
            "max_task_memory_gb": max(t.memory_required for t in tasks),
            "unique_params": len(params),
            "param_memory_gb": len(params) * param_cost,
            "sequential_compute_s": sum(t.compute_time for t in tasks),
            "max_dependencies": max(len(t.dependencies) for t in tasks),
            "avg_dependencies": float(np.mean([len(t.dependencies) for t in tasks])),
        }
        if verbose:
            print("DAG Analysis:")
            print(f"Total tasks: {info['total_tasks']}")
            print(f"Total memory (if sequential): {info['total_memory_gb']:.2f} GB")
            print(f"Max single task memory: {info['max_task_memory_gb']:.2f} GB")
            print(f"Unique parameters: {info['unique_params']}")
            print(f"Parameter memory: {info['param_memory_gb']:.2f} GB")
            print(f"Total compute time (sequential): {info['sequential_compute_s']:.2f} seconds")
            print(f"Max dependencies: {info['max_dependencies']}")
            print(f"Avg dependencies: {info['avg_dependencies']:.2f}")
        return info
