"""Plain PyTorch fp32 reference forwards over a :class:`ParamStore`.

These define what the DAG executor must produce (same weights, same tokens) and are
independent of the DAG machinery: a straight-line forward pass written from the model
definitions (GPT-2: pre-LN blocks, tanh-GELU MLP, tied LM head; Llama: RMSNorm, RoPE,
GQA, SwiGLU; Mixtral: top-k routed SwiGLU experts).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .config import ModelConfig
from .params import ParamStore


def _w(store: ParamStore, name: str) -> torch.Tensor:
    return store.tensor(name).float()


def _attn(q, k, v, nh, nkv, D, causal=True):
    B, S = q.shape[0], q.shape[1]
    q = q.view(B, S, nh, D).transpose(1, 2)
    k = k.view(B, S, nkv, D).transpose(1, 2)
    v = v.view(B, S, nkv, D).transpose(1, 2)
    if nh != nkv:
        k = k.repeat_interleave(nh // nkv, 1)
        v = v.repeat_interleave(nh // nkv, 1)
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, nh * D)


@torch.no_grad()
def gpt2_forward(cfg: ModelConfig, store: ParamStore, tokens: torch.Tensor, hidden: list = None) -> torch.Tensor:
    """tokens [B, S] -> logits [B, S, V] (fp32). ``hidden`` (if a list) receives the residual
    stream after every block."""
    B, S = tokens.shape
    H, nh = cfg.n_embd, cfg.n_head
    x = _w(store, "wte")[tokens.long()] + _w(store, "wpe")[:S][None]
    for i in range(cfg.n_layer):
        p = f"h.{i}."
        h = F.layer_norm(x, (H,), _w(store, p + "ln_1.weight"), _w(store, p + "ln_1.bias"), cfg.norm_eps)
        qkv = h @ _w(store, p + "attn.c_attn.weight").t() + _w(store, p + "attn.c_attn.bias")
        a = _attn(qkv[..., :H], qkv[..., H:2 * H], qkv[..., 2 * H:], nh, nh, cfg.head_dim)
        x = x + a @ _w(store, p + "attn.c_proj.weight").t() + _w(store, p + "attn.c_proj.bias")
        h = F.layer_norm(x, (H,), _w(store, p + "ln_2.weight"), _w(store, p + "ln_2.bias"), cfg.norm_eps)
        h = F.gelu(h @ _w(store, p + "mlp.c_fc.weight").t() + _w(store, p + "mlp.c_fc.bias"), approximate="tanh")
        x = x + h @ _w(store, p + "mlp.c_proj.weight").t() + _w(store, p + "mlp.c_proj.bias")
        if hidden is not None:
            hidden.append(x.clone())
    x = F.layer_norm(x, (H,), _w(store, "ln_f.weight"), _w(store, "ln_f.bias"), cfg.norm_eps)
    return x @ _w(store, "wte").t()


def _rope(x, S, D, theta):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None]
    c, s = ang.cos().float(), ang.sin().float()
    B = x.shape[0]
    x = x.view(B, S, -1, D)
    x1, x2 = x[..., :D // 2], x[..., D // 2:]
    c, s = c[None, :, None, :], s[None, :, None, :]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).view(B, S, -1)


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


@torch.no_grad()
def llama_forward(cfg: ModelConfig, store: ParamStore, tokens: torch.Tensor, router_margins: list = None) -> torch.Tensor:
    """Llama-3 / Mixtral forward (fp32): tokens [B, S] -> logits [B, S, V]. ``router_margins``
    (if a list) receives, per MoE layer, the [B, S] gap between the k-th and (k+1)-th router
    logit: tokens with a tiny gap may legitimately route differently under bf16 logits."""
    B, S = tokens.shape
    nh, nkv, D = cfg.n_head, cfg.kv_heads, cfg.head_dim
    x = _w(store, "tok_embeddings")[tokens.long()]
    for i in range(cfg.n_layer):
        p = f"layers.{i}."
        h = _rms(x, _w(store, p + "attention_norm.weight"), cfg.norm_eps)
        qkv = h @ _w(store, p + "attention.wqkv").t()
        q, k, v = qkv[..., :nh * D], qkv[..., nh * D:(nh + nkv) * D], qkv[..., (nh + nkv) * D:]
        q, k = _rope(q, S, D, cfg.rope_theta), _rope(k, S, D, cfg.rope_theta)
        x = x + _attn(q, k, v, nh, nkv, D) @ _w(store, p + "attention.wo").t()
        h = _rms(x, _w(store, p + "ffn_norm.weight"), cfg.norm_eps)
        if cfg.n_experts:
            logits = h @ _w(store, p + "moe.gate").t()
            val, idx = torch.topk(logits, cfg.top_k, -1)
            if router_margins is not None:
                srt = torch.sort(logits, -1, descending=True).values
                router_margins.append(srt[..., cfg.top_k - 1] - srt[..., cfg.top_k])
            gate = torch.softmax(val, -1)
            out = torch.zeros_like(h)
            for e in range(cfg.n_experts):
                gu = h @ _w(store, p + f"moe.experts.{e}.w13").t()
                y = F.silu(gu[..., :cfg.ffn]) * gu[..., cfg.ffn:]
                y = y @ _w(store, p + f"moe.experts.{e}.w2").t()
                wgt = (gate * (idx == e)).sum(-1, keepdim=True)
                out = out + wgt * y
            x = x + out
        else:
            gu = h @ _w(store, p + "feed_forward.w13").t()
            x = x + (F.silu(gu[..., :cfg.ffn]) * gu[..., cfg.ffn:]) @ _w(store, p + "feed_forward.w2").t()
    x = _rms(x, _w(store, "norm.weight"), cfg.norm_eps)
    return x @ _w(store, "output.weight").t()


def forward(cfg: ModelConfig, store: ParamStore, tokens: torch.Tensor, router_margins: list = None) -> torch.Tensor:
    if cfg.family == "gpt2":
        return gpt2_forward(cfg, store, tokens)
    return llama_forward(cfg, store, tokens, router_margins)
