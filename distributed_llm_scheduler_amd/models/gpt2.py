"""GPT-2 operator DAG (the reference's "real model" workload).

``build_gpt2_dag`` emits exactly the reference extractor's graph
(``/root/reference/test_gpt2.py:45-168``): ``embedding``, then per layer
``ln1 → attention → attn_residual(+prev) → ln2 → ffn_expand → ffn_activation →
ffn_contract → output(+attn_residual)``, then ``final_ln`` and a weight-tied
``output_projection`` — 1 + 8·L + 2 tasks (99 for gpt2-small), 6·L + 3 parameter ids
(75). With ``cost_model="reference"`` memory/compute numbers equal the reference's
(0.5 GB per parameter is applied by the scheduler; activation estimates follow its
``estimate_memory_gb`` formula, evaluated analytically from the config so no
``GPT2Model`` / network is needed). ``cost_model="bytes"`` uses real bf16 sizes and a
MI355X roofline for time.

Unlike the reference every task carries an :class:`OpSpec`, so the executor can run it.
"""
from __future__ import annotations

from typing import Dict, List

from ..core.task import OpSpec, Task
from .config import ModelConfig, get_config
from .params import ParamGroup, TensorSpec

# MI355X roofline used by the "bytes" cost model (dense bf16 MFMA peak is ~2.5 PF/s;
# ~40% is what small-M GEMMs reach; ~5 TB/s achievable HBM; ~3 us per kernel).
PEAK_FLOPS = 2.5e15 * 0.4
HBM_BW = 5.0e12
LAUNCH_S = 3e-6


# Logits rows are stored with their stride padded to a multiple of 64 columns (50257 ->
# 50304): 16-B aligned rows let the LM-head GEMM epilogue use vector stores. The logical
# shape stays [B, S, V]; the executor exposes a strided view.
LOGITS_PAD = 64


def _padded_cols(op) -> int:
    n = op.out_shape[-1]
    pad = op.attrs.get("ld_pad", 1)
    return (n + pad - 1) // pad * pad


def gpt2_param_groups(cfg: ModelConfig) -> Dict[str, ParamGroup]:
    H, V, F = cfg.n_embd, cfg.vocab_size, cfg.ffn
    g: Dict[str, ParamGroup] = {
        "embedding_weights": ParamGroup("embedding_weights", [TensorSpec("wte", (V, H))]),
        "position_weights": ParamGroup("position_weights", [TensorSpec("wpe", (cfg.n_positions, H), std=0.01)]),
    }
    for i in range(cfg.n_layer):
        p = f"h.{i}."
        g[f"layer_{i}_ln1_weights"] = ParamGroup(f"layer_{i}_ln1_weights", [
            TensorSpec(p + "ln_1.weight", (H,), "ln"), TensorSpec(p + "ln_1.bias", (H,), "bias")])
        g[f"layer_{i}_attn_qkv_weights"] = ParamGroup(f"layer_{i}_attn_qkv_weights", [
            TensorSpec(p + "attn.c_attn.weight", (3 * H, H)), TensorSpec(p + "attn.c_attn.bias", (3 * H,), "bias")])
        g[f"layer_{i}_attn_proj_weights"] = ParamGroup(f"layer_{i}_attn_proj_weights", [
            TensorSpec(p + "attn.c_proj.weight", (H, H)), TensorSpec(p + "attn.c_proj.bias", (H,), "bias")])
        g[f"layer_{i}_ln2_weights"] = ParamGroup(f"layer_{i}_ln2_weights", [
            TensorSpec(p + "ln_2.weight", (H,), "ln"), TensorSpec(p + "ln_2.bias", (H,), "bias")])
        g[f"layer_{i}_ffn_expand_weights"] = ParamGroup(f"layer_{i}_ffn_expand_weights", [
            TensorSpec(p + "mlp.c_fc.weight", (F, H)), TensorSpec(p + "mlp.c_fc.bias", (F,), "bias")])
        g[f"layer_{i}_ffn_contract_weights"] = ParamGroup(f"layer_{i}_ffn_contract_weights", [
            TensorSpec(p + "mlp.c_proj.weight", (H, F)), TensorSpec(p + "mlp.c_proj.bias", (H,), "bias")])
    g["final_ln_weights"] = ParamGroup("final_ln_weights", [
        TensorSpec("ln_f.weight", (H,), "ln"), TensorSpec("ln_f.bias", (H,), "bias")])
    return g


def _ref_estimate(n_params: int, weight_numel: int = 0) -> float:
    """The reference's estimate_memory_gb: fp32 params + (weight numel x batch(=1) x 4 B)
    if the module has a ``.weight``, else a flat 0.1 GB (test_gpt2.py:18-31)."""
    p = (n_params * 4) / 1e9
    a = (weight_numel * 1 * 4) / 1e9 if weight_numel else 0.1
    return p + a


def _roofline(flops: float, bytes_moved: float) -> float:
    return max(flops / PEAK_FLOPS, bytes_moved / HBM_BW) + LAUNCH_S


def build_gpt2_dag(cfg: "ModelConfig | str" = "gpt2", batch: int = 1, seq: int = 512,
                   cost_model: str = "reference", dtype_bytes: int = 2, prefix: str = "") -> List[Task]:
    """Return the GPT-2 task list. ``prefix`` namespaces task ids (used to instantiate
    several request replicas in one DAG; parameter ids stay shared)."""
    if isinstance(cfg, str):
        cfg = get_config(cfg)
    if cost_model not in ("reference", "bytes"):
        raise ValueError(f"cost_model must be 'reference' or 'bytes', got {cost_model!r}")
    H, V, F, L, nh = cfg.n_embd, cfg.vocab_size, cfg.ffn, cfg.n_layer, cfg.n_head
    M = batch * seq
    act = M * H * dtype_bytes
    groups = gpt2_param_groups(cfg)
    pbytes = {k: v.nbytes(dtype_bytes) for k, v in groups.items()}
    ref = cost_model == "reference"
    tid = (lambda s: prefix + s)
    tasks: List[Task] = []

    def add(name, mem_ref, t_ref, deps, params, op, flops, extra_bytes=0):
        out_b = dtype_bytes
        for s in op.out_shape[:-1]:
            out_b *= s
        out_b *= _padded_cols(op)
        if ref:
            mem, comp = mem_ref, t_ref
        else:
            moved = out_b + sum(pbytes[p] for p in params) + extra_bytes
            mem, comp = (out_b + extra_bytes) / 1e9, _roofline(flops, moved)
        tasks.append(Task(tid(name), mem, comp, [tid(d) for d in deps], set(params), op, out_b, flops))

    emb_mem = _ref_estimate(V * H, V * H)
    attn_mem = _ref_estimate(H * 3 * H + 3 * H + H * H + H)
    fc_mem = _ref_estimate(H * F + F, H * F)
    shape = (batch, seq, H)
    add("embedding", emb_mem, 0.1, [], ["embedding_weights", "position_weights"],
        OpSpec("embedding", [tid("@tokens")], {"wte": "wte", "wpe": "wpe"}, {"hidden": H}, shape), 0.0)
    for i in range(L):
        prev = "embedding" if i == 0 else f"layer_{i - 1}_output"
        p = f"h.{i}."
        add(f"layer_{i}_ln1", 0.01, 0.01, [prev], [f"layer_{i}_ln1_weights"],
            OpSpec("layernorm", [tid(prev)], {"w": p + "ln_1.weight", "b": p + "ln_1.bias"},
                   {"eps": cfg.norm_eps}, shape), 8.0 * M * H)
        qkv_f = 2.0 * M * H * 3 * H
        core_f = 2.0 * batch * nh * seq * seq * cfg.head_dim  # causal: half of 4*S^2*D per head
        proj_f = 2.0 * M * H * H
        add(f"layer_{i}_attention", attn_mem, 0.05, [f"layer_{i}_ln1"],
            [f"layer_{i}_attn_qkv_weights", f"layer_{i}_attn_proj_weights"],
            OpSpec("attention", [tid(f"layer_{i}_ln1")],
                   {"w_qkv": p + "attn.c_attn.weight", "b_qkv": p + "attn.c_attn.bias",
                    "w_o": p + "attn.c_proj.weight", "b_o": p + "attn.c_proj.bias"},
                   {"n_head": nh, "n_kv_head": nh, "head_dim": cfg.head_dim, "causal": True, "rope": False},
                   shape), qkv_f + core_f + proj_f, extra_bytes=3 * act)
        add(f"layer_{i}_attn_residual", 0.01, 0.01, [f"layer_{i}_attention", prev], [],
            OpSpec("residual", [tid(f"layer_{i}_attention"), tid(prev)], {}, {}, shape), 1.0 * M * H)
        add(f"layer_{i}_ln2", 0.01, 0.01, [f"layer_{i}_attn_residual"], [f"layer_{i}_ln2_weights"],
            OpSpec("layernorm", [tid(f"layer_{i}_attn_residual")], {"w": p + "ln_2.weight", "b": p + "ln_2.bias"},
                   {"eps": cfg.norm_eps}, shape), 8.0 * M * H)
        add(f"layer_{i}_ffn_expand", fc_mem, 0.08, [f"layer_{i}_ln2"], [f"layer_{i}_ffn_expand_weights"],
            OpSpec("linear", [tid(f"layer_{i}_ln2")], {"w": p + "mlp.c_fc.weight", "b": p + "mlp.c_fc.bias"},
                   {"act": None}, (batch, seq, F)), 2.0 * M * H * F)
        add(f"layer_{i}_ffn_activation", 0.01, 0.01, [f"layer_{i}_ffn_expand"], [],
            OpSpec("gelu", [tid(f"layer_{i}_ffn_expand")], {}, {"approximate": "tanh"}, (batch, seq, F)),
            8.0 * M * F)
        add(f"layer_{i}_ffn_contract", fc_mem, 0.08, [f"layer_{i}_ffn_activation"],
            [f"layer_{i}_ffn_contract_weights"],
            OpSpec("linear", [tid(f"layer_{i}_ffn_activation")],
                   {"w": p + "mlp.c_proj.weight", "b": p + "mlp.c_proj.bias"}, {"act": None}, shape),
            2.0 * M * H * F)
        add(f"layer_{i}_output", 0.01, 0.01, [f"layer_{i}_ffn_contract", f"layer_{i}_attn_residual"], [],
            OpSpec("residual", [tid(f"layer_{i}_ffn_contract"), tid(f"layer_{i}_attn_residual")], {}, {}, shape),
            1.0 * M * H)
    last = f"layer_{L - 1}_output"
    add("final_ln", 0.01, 0.01, [last], ["final_ln_weights"],
        OpSpec("layernorm", [tid(last)], {"w": "ln_f.weight", "b": "ln_f.bias"}, {"eps": cfg.norm_eps}, shape),
        8.0 * M * H)
    add("output_projection", emb_mem, 0.1, ["final_ln"], ["embedding_weights"],
        OpSpec("lm_head", [tid("final_ln")], {"w": "wte"}, {"vocab": V, "ld_pad": LOGITS_PAD}, (batch, seq, V)), 2.0 * M * H * V)
    return tasks


def build_replicated_dag(cfg="gpt2", replicas: int = 1, **kw) -> List[Task]:
    """``replicas`` independent request DAGs (ids prefixed ``r{k}/``) sharing parameter ids —
    the multi-request workload whose placement the schedulers decide (data parallelism
    expressed as a DAG)."""
    out: List[Task] = []
    for r in range(replicas):
        out.extend(build_gpt2_dag(cfg, prefix=f"r{r}/" if replicas > 1 else "", **kw))
    return out
