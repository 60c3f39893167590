"""DAG / placement checkpointing: JSON export/import of the task graph (with op specs) and
of a scheduling result, so a planned placement can be saved and replayed later without
re-running the policy (the reference only pickles the task list, test_gpt2.py:266-269)."""
from __future__ import annotations

import json
from typing import Dict, List, Sequence

from ..core.task import Task

FORMAT = "dlsched-dag/1"


def dag_to_dict(tasks: Sequence[Task]) -> Dict:
    return {"format": FORMAT, "tasks": [t.to_dict() for t in tasks]}


def dag_from_dict(d: Dict) -> List[Task]:
    if d.get("format") != FORMAT:
        raise ValueError(f"unsupported DAG format {d.get('format')!r}")
    return [Task.from_dict(x) for x in d["tasks"]]


def save_dag_json(tasks: Sequence[Task], path: str) -> None:
    with open(path, "w") as f:
        json.dump(dag_to_dict(tasks), f, indent=1)


def load_dag_json(path: str) -> List[Task]:
    with open(path) as f:
        return dag_from_dict(json.load(f))


def save_placement(path: str, schedule: Dict[str, List[str]], events: Sequence[tuple], nodes: Dict[str, Dict],
                   meta: Dict = None) -> None:
    """Persist a scheduling decision: per-node task order, the action trace and node specs."""
    with open(path, "w") as f:
        json.dump({"format": "dlsched-placement/1", "schedule": schedule, "events": [list(e) for e in events],
                   "nodes": nodes, "meta": meta or {}}, f, indent=1)


def load_placement(path: str) -> Dict:
    with open(path) as f:
        d = json.load(f)
    if d.get("format") != "dlsched-placement/1":
        raise ValueError("not a placement file")
    d["events"] = [tuple(e) for e in d["events"]]
    return d
