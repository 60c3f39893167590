"""Figures: the evaluation 2x2 panel, DAG drawings and Gantt charts.

Reference-compatible (``/root/reference/simulation.py:448-514``, ``visu.py:87-248``), with
two differences: figures are written to files (the reference only calls ``plt.show()``
though its README promises saved images), and the Gantt chart has a dependency-aware mode
plus a *measured* mode fed by the executor's per-kernel hipEvent timeline.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import matplotlib

if os.environ.get("DISPLAY") is None:
    matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

PALETTE = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f"]


def _finish(path: Optional[str], show: bool) -> None:
    plt.tight_layout()
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        plt.savefig(path, dpi=150 if not path.endswith("scheduler_performance.png") else 300, bbox_inches="tight")
    if show:
        plt.show()
    plt.close()


def performance_figure(df, path: Optional[str] = None, show: bool = False) -> None:
    """(a) completion vs memory regime, all DAGs; (b) same for LLM DAGs; (c) mean makespan
    by DAG type (rows with completed tasks); (d) load balance vs regime."""
    plt.figure(figsize=(12, 8))
    plt.subplot(2, 2, 1)
    comp = df.groupby(["scheduler_name", "memory_regime"])["completion_rate"].mean().reset_index()
    for s in df["scheduler_name"].unique():
        d = comp[comp["scheduler_name"] == s]
        plt.plot(d["memory_regime"] * 100, d["completion_rate"], marker="o", label=s, linewidth=2)
    plt.xlabel("Memory Regime (%)")
    plt.ylabel("Completion Rate (%)")
    plt.title("Average Task Completion Rate vs Memory Constraints")
    plt.legend()
    plt.grid(True, alpha=0.3)
    plt.subplot(2, 2, 2)
    llm = df[df["dag_type"].str.startswith("LLM")]
    lc = llm.groupby(["scheduler_name", "memory_regime"])["completion_rate"].mean().reset_index()
    for s in df["scheduler_name"].unique():
        d = lc[lc["scheduler_name"] == s]
        if not d.empty:
            plt.plot(d["memory_regime"] * 100, d["completion_rate"], marker="s", label=s, linewidth=2)
    plt.xlabel("Memory Regime (%)")
    plt.ylabel("Completion Rate (%)")
    plt.title("LLM DAG Completion Rate vs Memory Constraints")
    plt.legend()
    plt.grid(True, alpha=0.3)
    plt.subplot(2, 2, 3)
    done = df[df["completed_tasks"] > 0]
    if not done.empty:
        mk = done.groupby(["scheduler_name", "dag_type"])["makespan"].mean().reset_index()
        mk.pivot(index="dag_type", columns="scheduler_name", values="makespan").plot(kind="bar", ax=plt.gca())
        plt.ylabel("Makespan (seconds)")
        plt.xlabel("DAG Type")
        plt.title("Average Makespan by DAG Type (Completed Tasks Only)")
        plt.xticks(rotation=45)
        plt.legend(bbox_to_anchor=(1.05, 1), loc="upper left")
    plt.subplot(2, 2, 4)
    lb = done.groupby(["scheduler_name", "memory_regime"])["load_balance_score"].mean().reset_index()
    for s in df["scheduler_name"].unique():
        d = lb[lb["scheduler_name"] == s]
        if not d.empty:
            plt.plot(d["memory_regime"] * 100, d["load_balance_score"], marker="^", label=s, linewidth=2)
    plt.xlabel("Memory Regime (%)")
    plt.ylabel("Load Balance Score (0-1)")
    plt.title("Load Balance Quality vs Memory Constraints")
    plt.legend()
    plt.grid(True, alpha=0.3)
    _finish(path, show)


def _graph(tasks):
    import networkx as nx

    G = nx.DiGraph()
    for t in tasks:
        G.add_node(t.id)
        for d in t.dependencies:
            G.add_edge(d, t.id)
    return G


def visualize_dag_simple(tasks, title: str = "Task DAG", path: Optional[str] = None, show: bool = False) -> None:
    import networkx as nx

    G = _graph(tasks)
    plt.figure(figsize=(10, 8))
    pos = nx.spring_layout(G, k=3, iterations=50, seed=0) if len(tasks) < 10 else nx.spring_layout(G, seed=0)
    nx.draw(G, pos, with_labels=True, node_color="lightblue", node_size=1500, font_size=10, font_weight="bold",
            arrows=True, arrowsize=20, edge_color="gray", arrowstyle="->")
    plt.title(title, fontsize=16)
    plt.axis("off")
    _finish(path, show)


def _layer_index(tid: str) -> Optional[int]:
    base = tid.split("/")[-1]
    parts = base.split("_")
    if len(parts) > 1 and parts[0] == "layer" and parts[1].isdigit():
        return int(parts[1])
    return None


def visualize_dag_detailed(tasks, title: str = "Task DAG", path: Optional[str] = None, show: bool = False) -> None:
    """Colour = memory, size = compute time; LLM DAGs get one shell per layer (exact layer
    parsing — the reference's substring match merges layer_1 with layer_10..19)."""
    import networkx as nx

    G = _graph(tasks)
    tmap = {t.id: t for t in tasks}
    plt.figure(figsize=(12, 10))
    layers = {}
    for t in tasks:
        li = _layer_index(t.id)
        if li is not None:
            layers.setdefault(li, []).append(t.id)
    if layers:
        shells = []
        heads = [t.id for t in tasks if _layer_index(t.id) is None and not t.dependencies]
        if heads:
            shells.append(heads)
        shells += [layers[k] for k in sorted(layers)]
        tails = [t.id for t in tasks if _layer_index(t.id) is None and t.dependencies]
        if tails:
            shells.append(tails)
        pos = nx.shell_layout(G, shells)
    else:
        pos = nx.spring_layout(G, k=2, iterations=50, seed=0)
    colors = [tmap[n].memory_required for n in G.nodes()]
    sizes = [1000 + tmap[n].compute_time * 3000 for n in G.nodes()]
    vmax = max(colors) if colors else 1
    nx.draw_networkx_nodes(G, pos, node_color=colors, node_size=sizes, cmap="YlOrRd", vmin=0, vmax=vmax)
    nx.draw_networkx_edges(G, pos, edge_color="gray", arrows=True, arrowsize=20, alpha=0.6, arrowstyle="->")
    labels = {n: f"{n}\n{tmap[n].memory_required:.1f}GB\n{tmap[n].compute_time:.2f}s" for n in G.nodes()}
    nx.draw_networkx_labels(G, pos, labels, font_size=8)
    sm = plt.cm.ScalarMappable(cmap="YlOrRd", norm=plt.Normalize(vmin=0, vmax=vmax))
    sm.set_array([])
    plt.colorbar(sm, ax=plt.gca(), label="Memory Required (GB)")
    plt.title(f"{title}\nNode size = compute time, Color = memory requirement", fontsize=14)
    plt.axis("off")
    _finish(path, show)


def schedule_intervals(schedule: Dict[str, List[str]], tasks, nodes, respect_deps: bool = False
                       ) -> Dict[str, List[Tuple[str, float, float]]]:
    """Per-node (task, start, end) from a placement. ``respect_deps=False`` reproduces the
    reference's back-to-back layout (visu.py:220-238); True starts a task only after its
    dependencies finish (the honest timeline)."""
    tmap = {t.id: t for t in tasks}
    speed = {n.id: n.compute_speed for n in nodes}
    out: Dict[str, List[Tuple[str, float, float]]] = {n: [] for n in schedule}
    if not respect_deps:
        for nid, tids in schedule.items():
            now = 0.0
            for tid in tids:
                if tid in tmap:
                    d = tmap[tid].compute_time / speed[nid]
                    out[nid].append((tid, now, now + d))
                    now += d
        return out
    finish: Dict[str, float] = {}
    head = {n: 0 for n in schedule}
    free = {n: 0.0 for n in schedule}
    progress = True
    while progress:
        progress = False
        for nid, tids in schedule.items():
            while head[nid] < len(tids):
                t = tmap[tids[head[nid]]]
                if any(d not in finish for d in t.dependencies if d in tmap):
                    break
                st = max([free[nid]] + [finish[d] for d in t.dependencies if d in finish])
                finish[t.id] = st + t.compute_time / speed[nid]
                out[nid].append((t.id, st, finish[t.id]))
                free[nid] = finish[t.id]
                head[nid] += 1
                progress = True
    return out


def gantt(intervals: Dict[str, List[Tuple[str, float, float]]], node_labels: Optional[Dict[str, str]] = None,
          title: str = "Task Schedule Gantt Chart", xlabel: str = "Time (seconds)", path: Optional[str] = None,
          show: bool = False, label_tasks: bool = True) -> None:
    plt.figure(figsize=(12, max(3, 1.0 + 0.9 * len(intervals))))
    ylabels = []
    for y, (nid, items) in enumerate(intervals.items()):
        color = PALETTE[y % len(PALETTE)]
        for tid, a, b in items:
            plt.barh(y, b - a, left=a, height=0.8, color=color, edgecolor="black", linewidth=0.5)
            if label_tasks:
                plt.text(a + (b - a) / 2, y, tid.split("/")[-1], ha="center", va="center", fontsize=7, color="white",
                         weight="bold")
        ylabels.append(node_labels.get(nid, nid) if node_labels else nid)
    plt.yticks(range(len(ylabels)), ylabels)
    plt.xlabel(xlabel, fontsize=12)
    plt.title(title, fontsize=14)
    plt.grid(True, axis="x", alpha=0.3)
    _finish(path, show)


def visualize_schedule_simple(schedule: Dict[str, List[str]], tasks, nodes, path: Optional[str] = None,
                              show: bool = False, respect_deps: bool = False) -> None:
    """Reference-compatible Gantt (one row per node labelled ``id\\n(X.XGB)``)."""
    labels = {n.id: f"{n.id}\n({n.total_memory:.1f}GB)" for n in nodes}
    gantt(schedule_intervals(schedule, tasks, nodes, respect_deps), labels, path=path, show=show)


def measured_gantt(timelines: Dict[int, List[Tuple[str, float, float]]], path: Optional[str] = None,
                   show: bool = False, title: str = "Measured per-GPU kernel timeline (MI355X)") -> None:
    """Gantt of what the executor actually ran: rank -> [(task, start_ms, end_ms)]."""
    ivs = {f"GPU {r}": items for r, items in sorted(timelines.items())}
    gantt(ivs, title=title, xlabel="Time (ms)", path=path, show=show, label_tasks=False)
