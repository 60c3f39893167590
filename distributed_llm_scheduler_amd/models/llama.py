"""Llama-3 and Mixtral operator DAGs (BASELINE.json configs: Llama-3-8B pipeline-placed on
8 GPUs, Mixtral-8x7B with expert nodes spread over 8 GPUs under the 288 GB cap).

Per layer (ids follow the GPT-2 builder's naming so tooling is shared):

    attn_norm(rmsnorm) -> attention(GQA + RoPE) -> attn_residual(+prev) -> ffn_norm(rmsnorm)
      dense : -> mlp(SwiGLU: w13 -> silu*up -> w2) -> output(+attn_residual)
      MoE   : -> router(linear to E logits) -> expert_e (e = 0..E-1, top-k routed rows only)
              -> output(moe_combine: attn_residual + sum_e expert_e)

Expert-parallel placement is therefore a scheduling decision: each ``expert_e`` node is a
separate task with its own parameter group, and the router->expert / expert->combine
edges become RCCL transfers when the scheduler spreads experts over GPUs.
"""
from __future__ import annotations

from typing import Dict, List

from ..core.task import OpSpec, Task
from .config import ModelConfig, get_config
from .gpt2 import LOGITS_PAD, _padded_cols, _roofline
from .params import ParamGroup, TensorSpec


def llama_param_groups(cfg: ModelConfig) -> Dict[str, ParamGroup]:
    H, V, F = cfg.n_embd, cfg.vocab_size, cfg.ffn
    nh, nkv, D = cfg.n_head, cfg.kv_heads, cfg.head_dim
    g: Dict[str, ParamGroup] = {"embedding_weights": ParamGroup("embedding_weights", [TensorSpec("tok_embeddings",
                                                                                                 (V, H))])}
    for i in range(cfg.n_layer):
        p = f"layers.{i}."
        g[f"layer_{i}_attn_norm_weights"] = ParamGroup(f"layer_{i}_attn_norm_weights",
                                                       [TensorSpec(p + "attention_norm.weight", (H,), "ln")])
        g[f"layer_{i}_attn_qkv_weights"] = ParamGroup(f"layer_{i}_attn_qkv_weights",
                                                      [TensorSpec(p + "attention.wqkv", ((nh + 2 * nkv) * D, H))])
        g[f"layer_{i}_attn_proj_weights"] = ParamGroup(f"layer_{i}_attn_proj_weights",
                                                       [TensorSpec(p + "attention.wo", (H, nh * D))])
        g[f"layer_{i}_ffn_norm_weights"] = ParamGroup(f"layer_{i}_ffn_norm_weights",
                                                      [TensorSpec(p + "ffn_norm.weight", (H,), "ln")])
        if cfg.n_experts:
            g[f"layer_{i}_router_weights"] = ParamGroup(f"layer_{i}_router_weights",
                                                        [TensorSpec(p + "moe.gate", (cfg.n_experts, H))])
            for e in range(cfg.n_experts):
                q = p + f"moe.experts.{e}."
                g[f"layer_{i}_expert_{e}_weights"] = ParamGroup(f"layer_{i}_expert_{e}_weights", [
                    TensorSpec(q + "w13", (2 * F, H)), TensorSpec(q + "w2", (H, F))])
        else:
            g[f"layer_{i}_ffn_gate_up_weights"] = ParamGroup(f"layer_{i}_ffn_gate_up_weights",
                                                             [TensorSpec(p + "feed_forward.w13", (2 * F, H))])
            g[f"layer_{i}_ffn_down_weights"] = ParamGroup(f"layer_{i}_ffn_down_weights",
                                                          [TensorSpec(p + "feed_forward.w2", (H, F))])
    g["final_norm_weights"] = ParamGroup("final_norm_weights", [TensorSpec("norm.weight", (H,), "ln")])
    g["output_weights"] = ParamGroup("output_weights", [TensorSpec("output.weight", (V, H))])
    return g


def build_llama_dag(cfg: "ModelConfig | str" = "llama3-8b", batch: int = 1, seq: int = 512,
                    cost_model: str = "bytes", dtype_bytes: int = 2, prefix: str = "") -> List[Task]:
    if isinstance(cfg, str):
        cfg = get_config(cfg)
    H, V, F, L = cfg.n_embd, cfg.vocab_size, cfg.ffn, cfg.n_layer
    nh, nkv, D, E, K = cfg.n_head, cfg.kv_heads, cfg.head_dim, cfg.n_experts, cfg.top_k
    M = batch * seq
    groups = llama_param_groups(cfg)
    pbytes = {k: v.nbytes(dtype_bytes) for k, v in groups.items()}
    ref = cost_model == "reference"
    tid = (lambda s: prefix + s)
    tasks: List[Task] = []
    shape = (batch, seq, H)

    def add(name, t_ref, deps, params, op, flops, extra=0):
        out_b = dtype_bytes
        for s in op.out_shape[:-1]:
            out_b *= s
        out_b *= _padded_cols(op)
        if ref:
            mem = sum(pbytes[p] for p in params) * 2 / 1e9 + 0.01  # fp32 params + activation-ish, GPT-2 style
            comp = t_ref
        else:
            moved = out_b + sum(pbytes[p] for p in params) + extra
            mem, comp = (out_b + extra) / 1e9, _roofline(flops, moved)
        tasks.append(Task(tid(name), mem, comp, [tid(d) for d in deps], set(params), op, out_b, flops))

    add("embedding", 0.1, [], ["embedding_weights"],
        OpSpec("embedding", [tid("@tokens")], {"wte": "tok_embeddings"}, {"hidden": H}, shape), 0.0)
    attn_attrs = {"n_head": nh, "n_kv_head": nkv, "head_dim": D, "causal": True, "rope": True,
                  "rope_theta": cfg.rope_theta}
    for i in range(L):
        prev = "embedding" if i == 0 else f"layer_{i - 1}_output"
        p = f"layers.{i}."
        add(f"layer_{i}_attn_norm", 0.01, [prev], [f"layer_{i}_attn_norm_weights"],
            OpSpec("rmsnorm", [tid(prev)], {"w": p + "attention_norm.weight"}, {"eps": cfg.norm_eps}, shape),
            4.0 * M * H)
        fl = 2.0 * M * H * (nh + 2 * nkv) * D + 2.0 * batch * nh * seq * seq * D + 2.0 * M * nh * D * H
        add(f"layer_{i}_attention", 0.05, [f"layer_{i}_attn_norm"],
            [f"layer_{i}_attn_qkv_weights", f"layer_{i}_attn_proj_weights"],
            OpSpec("attention", [tid(f"layer_{i}_attn_norm")], {"w_qkv": p + "attention.wqkv", "w_o": p + "attention.wo"},
                   dict(attn_attrs), shape), fl, extra=M * (2 * nh + 2 * nkv) * D * dtype_bytes)
        add(f"layer_{i}_attn_residual", 0.01, [f"layer_{i}_attention", prev], [],
            OpSpec("residual", [tid(f"layer_{i}_attention"), tid(prev)], {}, {}, shape), 1.0 * M * H)
        add(f"layer_{i}_ffn_norm", 0.01, [f"layer_{i}_attn_residual"], [f"layer_{i}_ffn_norm_weights"],
            OpSpec("rmsnorm", [tid(f"layer_{i}_attn_residual")], {"w": p + "ffn_norm.weight"}, {"eps": cfg.norm_eps},
                   shape), 4.0 * M * H)
        if E:
            add(f"layer_{i}_router", 0.01, [f"layer_{i}_ffn_norm"], [f"layer_{i}_router_weights"],
                OpSpec("linear", [tid(f"layer_{i}_ffn_norm")], {"w": p + "moe.gate"}, {"act": None},
                       (batch, seq, E)), 2.0 * M * H * E)
            experts = []
            for e in range(E):
                q = p + f"moe.experts.{e}."
                rows = M * K / E  # expected routed rows per expert
                add(f"layer_{i}_expert_{e}", 0.08 * K / E, [f"layer_{i}_ffn_norm", f"layer_{i}_router"],
                    [f"layer_{i}_expert_{e}_weights"],
                    OpSpec("moe_expert", [tid(f"layer_{i}_ffn_norm"), tid(f"layer_{i}_router")],
                           {"w_gate_up": q + "w13", "w_down": q + "w2"},
                           {"expert": e, "n_experts": E, "top_k": K, "ffn": F}, shape),
                    6.0 * rows * H * F, extra=M * K * (H + 3 * F) * dtype_bytes)
                experts.append(f"layer_{i}_expert_{e}")
            # a cross-GPU edge into or out of an expert moves the whole [M, H] buffer (the normed
            # hidden state in, the expert's compact output rows back): fixed-size transfers that
            # need no routing on the host, so an expert-parallel step replays like any other
            # (each expert GPU routes locally from the router logits, which travel too). Per
            # expert GPU this is never more than the worst case of the routed rows
            # (M x min(top-k, experts there) rows).
            # combine = residual + gate-weighted gather of the experts' compact outputs; the
            # router edge carries the (tiny) logits so routing is known wherever this runs
            add(f"layer_{i}_output", 0.01, experts + [f"layer_{i}_router", f"layer_{i}_attn_residual"], [],
                OpSpec("moe_combine", [tid(x) for x in experts] + [tid(f"layer_{i}_router"),
                                                                   tid(f"layer_{i}_attn_residual")],
                       {}, {"n_experts": E, "top_k": K}, shape),
                1.0 * M * H * (K + 1))
        else:
            add(f"layer_{i}_mlp", 0.16, [f"layer_{i}_ffn_norm"],
                [f"layer_{i}_ffn_gate_up_weights", f"layer_{i}_ffn_down_weights"],
                OpSpec("swiglu_mlp", [tid(f"layer_{i}_ffn_norm")],
                       {"w_gate_up": p + "feed_forward.w13", "w_down": p + "feed_forward.w2"}, {"ffn": F}, shape),
                6.0 * M * H * F, extra=3 * M * F * dtype_bytes)
            add(f"layer_{i}_output", 0.01, [f"layer_{i}_mlp", f"layer_{i}_attn_residual"], [],
                OpSpec("residual", [tid(f"layer_{i}_mlp"), tid(f"layer_{i}_attn_residual")], {}, {}, shape),
                1.0 * M * H)
    last = f"layer_{L - 1}_output"
    add("final_ln", 0.01, [last], ["final_norm_weights"],
        OpSpec("rmsnorm", [tid(last)], {"w": "norm.weight"}, {"eps": cfg.norm_eps}, shape), 4.0 * M * H)
    add("output_projection", 0.1, ["final_ln"], ["output_weights"],
        OpSpec("lm_head", [tid("final_ln")], {"w": "output.weight"}, {"vocab": V, "ld_pad": LOGITS_PAD},
               (batch, seq, V)),
        2.0 * M * H * V)
    return tasks
