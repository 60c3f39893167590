"""Data model: tasks (DAG vertices) and nodes (devices).

Field names and constructor signatures match the reference so user code written for it
keeps working (``/root/reference/schedulers.py:7-29``):

* ``Task(task_id, memory_required, compute_time, dependencies=None, params_needed=None)``
  with mutable ``completed`` / ``assigned_node``.
* ``Node(node_id, total_memory, compute_speed=1.0)`` with ``available_memory``,
  ``cached_params``, ``running_tasks``, ``completed_tasks``, ``last_used_params``.

Additions for real execution (absent in the reference, which never runs anything):

* ``Task.op`` — an :class:`OpSpec` naming the kernel that implements the vertex, its
  input tensors (by producing task id) and the parameter tensors it reads.
* ``Task.out_bytes`` — bytes of the activation the task produces (the payload of every
  outgoing edge; crosses xGMI when the consumer sits on another GPU).
* ``Node.device`` — the GPU ordinal (rank) a node maps to in the executor.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple


@dataclass
class OpSpec:
    """What a DAG vertex computes.

    ``kind``    — kernel family, e.g. ``"embedding"``, ``"layernorm"``, ``"attention"``,
                  ``"linear"``, ``"gelu"``, ``"residual"``, ``"lm_head"``, ``"rmsnorm"``,
                  ``"swiglu_mlp"``, ``"moe_router"``, ``"moe_expert"``, ``"moe_combine"``.
    ``inputs``  — producing task ids whose outputs feed this op, in argument order.
    ``weights`` — mapping of role -> parameter-tensor name (e.g. ``{"w": "h.0.attn.c_attn.weight"}``).
    ``attrs``   — shapes/static attributes (eps, heads, activation, ...).
    ``out_shape`` — activation shape produced (per micro-batch), dtype in ``attrs["dtype"]``.
    """

    kind: str
    inputs: List[str] = field(default_factory=list)
    weights: Dict[str, str] = field(default_factory=dict)
    attrs: Dict[str, Any] = field(default_factory=dict)
    out_shape: Tuple[int, ...] = ()

    def to_dict(self) -> Dict[str, Any]:
        return {"kind": self.kind, "inputs": list(self.inputs), "weights": dict(self.weights),
                "attrs": dict(self.attrs), "out_shape": list(self.out_shape)}

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "OpSpec":
        return OpSpec(d["kind"], list(d.get("inputs", [])), dict(d.get("weights", {})),
                      dict(d.get("attrs", {})), tuple(d.get("out_shape", ())))


class Task:
    """A DAG vertex. ``memory_required`` in GB (freed at completion), ``compute_time`` in
    seconds on a speed-1.0 node, ``params_needed`` a set of parameter ids (persist in the
    node's cache after use)."""

    __slots__ = ("id", "memory_required", "compute_time", "dependencies", "params_needed",
                 "completed", "assigned_node", "op", "out_bytes", "flops", "edge_bytes")

    def __init__(self, task_id: str, memory_required: float, compute_time: float,
                 dependencies: Optional[List[str]] = None, params_needed: Optional[Set[str]] = None,
                 op: Optional[OpSpec] = None, out_bytes: int = 0, flops: float = 0.0,
                 edge_bytes: Optional[int] = None):
        self.id = task_id
        self.memory_required = memory_required
        self.compute_time = compute_time
        self.dependencies = dependencies or []
        self.params_needed = params_needed or set()
        self.completed = False
        self.assigned_node = None
        self.op = op
        self.out_bytes = out_bytes
        self.flops = flops
        # bytes one cross-GPU edge out of this task moves, when that is less than its whole
        # output buffer (``out_bytes``, the activation arena size): an MoE expert returns only
        # its routed rows, the routed hidden state ships each expert only its rows. Transfer
        # costs (EFT) use it; None = out_bytes
        self.edge_bytes = edge_bytes

    @property
    def xfer_bytes(self) -> int:
        return self.out_bytes if self.edge_bytes is None else self.edge_bytes

    def __repr__(self) -> str:
        return (f"Task({self.id!r}, mem={self.memory_required:.3f}GB, t={self.compute_time:.3f}s, "
                f"deps={self.dependencies}, params={sorted(self.params_needed)})")

    def __getstate__(self):
        return {k: getattr(self, k) for k in self.__slots__}

    def __setstate__(self, state):
        for k in self.__slots__:
            setattr(self, k, state.get(k))

    def clone(self) -> "Task":
        """Fresh, un-executed copy (the harness deep-copies before every run,
        ``/root/reference/simulation.py:308-317``)."""
        return Task(self.id, self.memory_required, self.compute_time, list(self.dependencies),
                    set(self.params_needed), self.op, self.out_bytes, self.flops, self.edge_bytes)

    def to_dict(self) -> Dict[str, Any]:
        return {"id": self.id, "memory_required": self.memory_required, "compute_time": self.compute_time,
                "dependencies": list(self.dependencies), "params_needed": sorted(self.params_needed),
                "out_bytes": int(self.out_bytes), "flops": float(self.flops),
                **({"edge_bytes": int(self.edge_bytes)} if self.edge_bytes is not None else {}),
                "op": self.op.to_dict() if self.op is not None else None}

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "Task":
        op = OpSpec.from_dict(d["op"]) if d.get("op") else None
        return Task(d["id"], d["memory_required"], d["compute_time"], list(d.get("dependencies", [])),
                    set(d.get("params_needed", [])), op, int(d.get("out_bytes", 0)), float(d.get("flops", 0.0)),
                    d.get("edge_bytes"))


class Node:
    """A device with a memory budget (GB) and a relative speed."""

    def __init__(self, node_id: str, total_memory: float, compute_speed: float = 1.0, device: Optional[int] = None):
        self.id = node_id
        self.total_memory = total_memory
        self.available_memory = total_memory
        self.compute_speed = compute_speed
        self.cached_params: Set[str] = set()
        self.running_tasks: List[str] = []
        self.completed_tasks: List[str] = []
        self.last_used_params = deque(maxlen=10)
        self.device = device

    def fresh(self) -> "Node":
        return Node(self.id, self.total_memory, self.compute_speed, self.device)

    def __repr__(self) -> str:
        return f"Node({self.id!r}, {self.total_memory:.3f}GB, speed={self.compute_speed:.2f})"


def clone_tasks(tasks: Sequence[Task]) -> List[Task]:
    return [t.clone() for t in tasks]


def clone_nodes(nodes: Sequence[Node]) -> List[Node]:
    return [n.fresh() for n in nodes]
