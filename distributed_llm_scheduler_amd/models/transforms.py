"""DAG transformations: tensor parallelism expressed in the task graph.

``tensor_parallel(tasks, groups, cfg, degree)`` rewrites every transformer layer so a
scheduler can spread one layer's work over ``degree`` GPUs (SURVEY §2.3 "TP: head-group
split attention nodes and column/row-split GEMM nodes as a DAG transformation"):

* attention -> ``degree`` head-group shards. Shard k owns q heads [k·nh/T, (k+1)·nh/T) and
  kv heads [k·nkv/T, ...): its QKV weight rows and its W_o columns (row-parallel output
  projection), producing a PARTIAL [B, S, H]; the output bias lives in shard 0 only.
* MLP -> column-parallel up-projection (+activation) and row-parallel down-projection
  per shard (GPT-2: fc1 rows / fc2 columns; Llama: SwiGLU gate+up rows / w2 columns).
* a ``sum`` node adds the shard partials (the "all-reduce" — its inputs arrive over xGMI
  as RCCL point-to-point edges when the shards sit on other GPUs), then the layer's
  residual node consumes it unchanged.
* the norm feeding a shard is replicated per shard (cheap, and lets every shard fold it
  into its first GEMM).

Shard weights are SLICES of the full tensors (``TensorSpec.parent``), so a TP execution is
numerically the same model as the unsharded one and checks against the same reference.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Tuple

from ..core.task import OpSpec, Task
from .config import ModelConfig
from .params import ParamGroup, TensorSpec


def _slice(spec: TensorSpec, dim: int, start: int, stop: int, tag: str) -> TensorSpec:
    shape = list(spec.shape)
    shape[dim] = stop - start
    return TensorSpec(f"{spec.name}.{tag}", tuple(shape), spec.init, spec.std, parent=spec, slc=(dim, start, stop))


def _rows(spec: TensorSpec, ranges: List[Tuple[int, int]], tag: str) -> TensorSpec:
    """Concatenation of row ranges of ``spec`` (e.g. the q, k and v rows of one head group)."""
    n = sum(b - a for a, b in ranges)
    return TensorSpec(f"{spec.name}.{tag}", (n,) + tuple(spec.shape[1:]), spec.init, spec.std, parent=spec,
                      slc=("rows", tuple(ranges)))


def tensor_parallel(tasks: List[Task], groups: Dict[str, ParamGroup], cfg: ModelConfig, degree: int
                    ) -> Tuple[List[Task], Dict[str, ParamGroup]]:
    T = degree
    if T <= 1:
        return tasks, groups
    nh, nkv, D, H, F = cfg.n_head, cfg.kv_heads, cfg.head_dim, cfg.n_embd, cfg.ffn
    if nh % T or nkv % T or F % T:
        raise ValueError(f"TP degree {T} must divide heads ({nh}), kv heads ({nkv}) and ffn ({F})")
    spec_of = {s.name: s for g in groups.values() for s in g.tensors}
    owner = {s.name: pid for pid, g in groups.items() for s in g.tensors}
    new_groups: Dict[str, ParamGroup] = dict(groups)
    out: List[Task] = []
    tmap = {t.id: t for t in tasks}
    consumers: Dict[str, List[str]] = {}
    for t in tasks:
        for d in t.dependencies:
            consumers.setdefault(d, []).append(t.id)
    replaced: Dict[str, str] = {}  # original task id -> id of the node that now provides its output
    hq, hkv, fs = nh // T, nkv // T, F // T

    def add_group(pid: str, specs: List[TensorSpec]) -> str:
        new_groups[pid] = ParamGroup(pid, specs)
        return pid

    def norm_copy(norm: Task, k: int) -> Task:
        n = copy.copy(norm)
        n.id = f"{norm.id}.tp{k}"
        n.op = copy.deepcopy(norm.op)
        n.params_needed = set(norm.params_needed)
        n.dependencies = list(norm.dependencies)
        return n

    skip = set()
    for t in tasks:
        if t.id in skip:
            continue
        kind = t.op.kind if t.op else ""
        # ---- attention: norm -> attention  ==>  T x (norm copy -> shard) -> sum
        if kind == "attention" and len(t.dependencies) == 1 and tmap[t.dependencies[0]].op.kind in (
                "layernorm", "rmsnorm") and len(consumers.get(t.dependencies[0], [])) == 1:
            norm = tmap[t.dependencies[0]]
            out = [x for x in out if x.id != norm.id]
            wq = spec_of[t.op.weights["w_qkv"]]
            wo = spec_of[t.op.weights["w_o"]]
            bq = spec_of.get(t.op.weights.get("b_qkv", ""))
            bo_name = t.op.weights.get("b_o")
            parts = []
            for k in range(T):
                qr = (k * hq * D, (k + 1) * hq * D)
                kr = (nh * D + k * hkv * D, nh * D + (k + 1) * hkv * D)
                vr = ((nh + nkv) * D + k * hkv * D, (nh + nkv) * D + (k + 1) * hkv * D)
                tag = f"tp{k}"
                g_qkv = [_rows(wq, [qr, kr, vr], tag)] + ([_rows(bq, [qr, kr, vr], tag)] if bq else [])
                pid_qkv = add_group(f"{owner[wq.name]}.{tag}", g_qkv)
                g_o = [_slice(wo, 1, k * hq * D, (k + 1) * hq * D, tag)]
                if bo_name and k == 0:
                    g_o.append(spec_of[bo_name])
                pid_o = add_group(f"{owner[wo.name]}.{tag}", g_o)
                nc = norm_copy(norm, k)
                out.append(nc)
                w = {"w_qkv": g_qkv[0].name, "w_o": g_o[0].name}
                if bq:
                    w["b_qkv"] = g_qkv[1].name
                if bo_name and k == 0:
                    w["b_o"] = bo_name
                attrs = dict(t.op.attrs, n_head=hq, n_kv_head=hkv)
                sh = Task(f"{t.id}.tp{k}", t.memory_required / T, t.compute_time / T, [nc.id],
                          {pid_qkv, pid_o}, OpSpec("attention", [nc.id], w, attrs, t.op.out_shape), t.out_bytes,
                          t.flops / T)
                out.append(sh)
                parts.append(sh.id)
            red = Task(f"{t.id}.sum", 0.01, 0.01, list(parts), set(), OpSpec("sum", list(parts), {}, {},
                                                                          t.op.out_shape), t.out_bytes, 0.0)
            out.append(red)
            replaced[t.id] = red.id
            continue
        # ---- GPT-2 MLP: norm -> linear(fc1) -> gelu -> linear(fc2)
        if kind == "linear" and len(t.dependencies) == 1 and tmap[t.dependencies[0]].op.kind == "layernorm" \
                and len(consumers.get(t.id, [])) == 1 and tmap[consumers[t.id][0]].op.kind == "gelu":
            norm = tmap[t.dependencies[0]]
            act = tmap[consumers[t.id][0]]
            if len(consumers.get(act.id, [])) != 1:
                out.append(t)
                continue
            fc2 = tmap[consumers[act.id][0]]
            if not (fc2.op and fc2.op.kind == "linear"):
                out.append(t)
                continue
            out = [x for x in out if x.id != norm.id]
            skip |= {act.id, fc2.id}
            w1, b1 = spec_of[t.op.weights["w"]], spec_of.get(t.op.weights.get("b", ""))
            w2, b2 = spec_of[fc2.op.weights["w"]], fc2.op.weights.get("b")
            parts = []
            for k in range(T):
                tag = f"tp{k}"
                g1 = [_slice(w1, 0, k * fs, (k + 1) * fs, tag)] + ([_slice(b1, 0, k * fs, (k + 1) * fs, tag)]
                                                                   if b1 else [])
                pid1 = add_group(f"{owner[w1.name]}.{tag}", g1)
                g2 = [_slice(w2, 1, k * fs, (k + 1) * fs, tag)] + ([spec_of[b2]] if (b2 and k == 0) else [])
                pid2 = add_group(f"{owner[w2.name]}.{tag}", g2)
                nc = norm_copy(norm, k)
                out.append(nc)
                fshape = t.op.out_shape[:-1] + (fs,)
                wd1 = {"w": g1[0].name}
                if b1:
                    wd1["b"] = g1[1].name
                up = Task(f"{t.id}.tp{k}", t.memory_required / T, t.compute_time / T, [nc.id], {pid1},
                          OpSpec("linear", [nc.id], wd1, dict(t.op.attrs), fshape), t.out_bytes // T, t.flops / T)
                ac = Task(f"{act.id}.tp{k}", act.memory_required / T, act.compute_time / T, [up.id], set(),
                          OpSpec("gelu", [up.id], {}, dict(act.op.attrs), fshape), act.out_bytes // T,
                          act.flops / T)
                wd2 = {"w": g2[0].name}
                if b2 and k == 0:
                    wd2["b"] = b2
                dn = Task(f"{fc2.id}.tp{k}", fc2.memory_required / T, fc2.compute_time / T, [ac.id], {pid2},
                          OpSpec("linear", [ac.id], wd2, dict(fc2.op.attrs), fc2.op.out_shape), fc2.out_bytes,
                          fc2.flops / T)
                out += [up, ac, dn]
                parts.append(dn.id)
            red = Task(f"{fc2.id}.sum", 0.01, 0.01, list(parts), set(),
                       OpSpec("sum", list(parts), {}, {}, fc2.op.out_shape), fc2.out_bytes, 0.0)
            out.append(red)
            replaced[fc2.id] = red.id
            continue
        # ---- Llama MLP: norm -> swiglu_mlp
        if kind == "swiglu_mlp" and len(t.dependencies) == 1 and tmap[t.dependencies[0]].op.kind == "rmsnorm" \
                and len(consumers.get(t.dependencies[0], [])) == 1:
            norm = tmap[t.dependencies[0]]
            out = [x for x in out if x.id != norm.id]
            w13, w2 = spec_of[t.op.weights["w_gate_up"]], spec_of[t.op.weights["w_down"]]
            parts = []
            for k in range(T):
                tag = f"tp{k}"
                g13 = _rows(w13, [(k * fs, (k + 1) * fs), (F + k * fs, F + (k + 1) * fs)], tag)
                g2 = _slice(w2, 1, k * fs, (k + 1) * fs, tag)
                pid1 = add_group(f"{owner[w13.name]}.{tag}", [g13])
                pid2 = add_group(f"{owner[w2.name]}.{tag}", [g2])
                nc = norm_copy(norm, k)
                out.append(nc)
                sh = Task(f"{t.id}.tp{k}", t.memory_required / T, t.compute_time / T, [nc.id], {pid1, pid2},
                          OpSpec("swiglu_mlp", [nc.id], {"w_gate_up": g13.name, "w_down": g2.name},
                                 dict(t.op.attrs, ffn=fs), t.op.out_shape), t.out_bytes, t.flops / T)
                out.append(sh)
                parts.append(sh.id)
            red = Task(f"{t.id}.sum", 0.01, 0.01, list(parts), set(),
                       OpSpec("sum", list(parts), {}, {}, t.op.out_shape), t.out_bytes, 0.0)
            out.append(red)
            replaced[t.id] = red.id
            continue
        out.append(t)
    # rewire consumers of replaced nodes (dependencies and op inputs)
    final: List[Task] = []
    for t in out:
        if any(d in replaced for d in t.dependencies):
            t = copy.copy(t)
            t.dependencies = [replaced.get(d, d) for d in t.dependencies]
            t.op = copy.deepcopy(t.op)
            t.op.inputs = [replaced.get(d, d) for d in t.op.inputs]
        final.append(t)
    # drop parameter groups no task references any more (the unsharded weights)
    used = set().union(*[t.params_needed for t in final])
    new_groups = {pid: g for pid, g in new_groups.items() if pid in used}
    return final, new_groups


def sequence_parallel(tasks: List[Task], groups: Dict[str, ParamGroup], cfg: ModelConfig, degree: int
                      ) -> Tuple[List[Task], Dict[str, ParamGroup]]:
    """Sequence (context) parallelism as a DAG transform: every token-wise node is split into
    ``degree`` sequence chunks (chunk c = positions [c*S/P, (c+1)*S/P) of every sequence, all
    batch rows), so a scheduler can place the chunks of one long request on different GPUs.

    Only attention mixes positions. Each attention node becomes, per chunk c,

    * ``...attention.qkv.sp{c}`` (``qkv_proj``) — the QKV projection of chunk c's rows (RoPE at
      the chunk's absolute positions), and
    * ``...attention.sp{c}`` (``attn_sp``) — chunk c's queries against the keys/values of
      chunks 0..c (causal; all chunks otherwise), then the output projection.

    So the K/V of chunk j flow along DAG edges qkv.sp{j} -> attention.sp{c>=j}: placed on
    different GPUs those edges are RCCL point-to-point transfers — ring attention expressed
    as DAG edges (SURVEY §2.3 "SP / CP", §5 "Long-context"). Weights are shared, so the
    transformed DAG is numerically the same model (the chunks' outputs concatenate to it).
    """
    P = degree
    if P <= 1:
        return tasks, groups
    owner = {s.name: pid for pid, g in groups.items() for s in g.tensors}
    ids = {t.id for t in tasks}
    out: List[Task] = []

    def chunk_id(name: str, c: int) -> str:
        return f"{name}.sp{c}" if name in ids else name  # external inputs (token ids) stay whole

    for t in tasks:
        if t.op is None or not t.op.out_shape or len(t.op.out_shape) != 3:
            raise ValueError(f"sequence_parallel: task {t.id} has no [B, S, X] output")
        B, S, X = t.op.out_shape
        if S % P:
            raise ValueError(f"sequence_parallel: degree {P} must divide the sequence length {S}")
        Sc = S // P
        kind = t.op.kind
        if kind == "attention":
            a = t.op.attrs
            nh, nkv, D = a["n_head"], a["n_kv_head"], a["head_dim"]
            width = (nh + 2 * nkv) * D
            wq = {k: v for k, v in t.op.weights.items() if k in ("w_qkv", "b_qkv")}
            wo = {k: v for k, v in t.op.weights.items() if k in ("w_o", "b_o")}
            pq = {owner[v] for v in wq.values()}
            po = {owner[v] for v in wo.values()}
            M = B * Sc
            qkv_f = 2.0 * M * X * width
            qkv_ids = []
            for c in range(P):
                src = chunk_id(t.op.inputs[0], c)
                q = Task(f"{t.id}.qkv.sp{c}", t.memory_required / (2 * P), t.compute_time / (2 * P), [src], set(pq),
                         OpSpec("qkv_proj", [src], dict(wq), dict(a, seq_chunk=(c, P)), (B, Sc, width)),
                         2 * M * width, qkv_f)
                out.append(q)
                qkv_ids.append(q.id)
            causal = a.get("causal", True)
            for c in range(P):
                kv = qkv_ids[:c + 1] if causal else list(qkv_ids)
                nkeys = len(kv) * Sc
                core_f = 2.0 * 2 * B * nh * Sc * nkeys * D / (2 if causal else 1) + 2.0 * M * nh * D * X
                at = Task(f"{t.id}.sp{c}", t.memory_required / (2 * P), t.compute_time * len(kv) / (P * P), kv,
                          set(po), OpSpec("attn_sp", kv, dict(wo), dict(a, seq_chunk=(c, P)), (B, Sc, X)),
                          t.out_bytes // P, core_f)
                out.append(at)
            continue
        for c in range(P):
            op = copy.deepcopy(t.op)
            op.inputs = [chunk_id(i, c) for i in op.inputs]
            op.out_shape = (B, Sc, X)
            if kind == "embedding":
                op.attrs = dict(op.attrs, seq_chunk=(c, P), tokens_total=B * S)
            out.append(Task(f"{t.id}.sp{c}", t.memory_required / P, t.compute_time / P,
                            [chunk_id(d, c) for d in t.dependencies], set(t.params_needed), op, t.out_bytes // P,
                            t.flops / P))
    return out, groups
