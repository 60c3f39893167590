"""Model presets (local — no Hub download; the reference's ``GPT2Config.from_pretrained``
needs the network, ``/root/reference/test_gpt2.py:47``).

GPT-2 numbers are ``transformers.GPT2Config()`` defaults (== the "gpt2" checkpoint's
config) and gpt2-medium's published config. Llama-3-8B / Mixtral-8x7B follow their public
model cards. ``tiny-*`` presets exist for CPU tests.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace
from typing import Dict


@dataclass(frozen=True)
class ModelConfig:
    name: str
    family: str  # "gpt2" | "llama" | "mixtral"
    n_layer: int
    n_embd: int
    n_head: int
    vocab_size: int
    n_positions: int = 1024
    ffn_dim: int = 0  # 0 -> 4 * n_embd
    n_kv_head: int = 0  # 0 -> n_head
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    n_experts: int = 0
    top_k: int = 0
    tie_embeddings: bool = True

    @property
    def ffn(self) -> int:
        return self.ffn_dim or 4 * self.n_embd

    @property
    def kv_heads(self) -> int:
        return self.n_kv_head or self.n_head

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    def with_(self, **kw) -> "ModelConfig":
        return replace(self, **kw)

    def to_dict(self) -> Dict:
        return asdict(self)


PRESETS: Dict[str, ModelConfig] = {
    "gpt2": ModelConfig("gpt2", "gpt2", 12, 768, 12, 50257),
    "gpt2-medium": ModelConfig("gpt2-medium", "gpt2", 24, 1024, 16, 50257),
    "gpt2-large": ModelConfig("gpt2-large", "gpt2", 36, 1280, 20, 50257),
    "llama3-8b": ModelConfig("llama3-8b", "llama", 32, 4096, 32, 128256, n_positions=8192, ffn_dim=14336,
                             n_kv_head=8, norm_eps=1e-5, rope_theta=500000.0, tie_embeddings=False),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", "mixtral", 32, 4096, 32, 32000, n_positions=32768, ffn_dim=14336,
                                n_kv_head=8, norm_eps=1e-5, rope_theta=1e6, n_experts=8, top_k=2,
                                tie_embeddings=False),
    # CPU-test sized variants (same structure, small dims)
    "tiny-gpt2": ModelConfig("tiny-gpt2", "gpt2", 2, 64, 4, 256, n_positions=128),
    "tiny-llama": ModelConfig("tiny-llama", "llama", 2, 64, 4, 256, n_positions=128, ffn_dim=128, n_kv_head=2,
                              tie_embeddings=False),
    "tiny-mixtral": ModelConfig("tiny-mixtral", "mixtral", 2, 64, 4, 256, n_positions=128, ffn_dim=96, n_kv_head=2,
                                n_experts=4, top_k=2, tie_embeddings=False),
    # smallest shapes the GPU kernels take (head_dim 64, 128-multiple GEMM dims): GPU tests
    "mini-gpt2": ModelConfig("mini-gpt2", "gpt2", 2, 256, 4, 1024, n_positions=256),
    "mini-llama": ModelConfig("mini-llama", "llama", 2, 256, 4, 1024, n_positions=256, ffn_dim=512, n_kv_head=2,
                              tie_embeddings=False),
    "mini-mixtral": ModelConfig("mini-mixtral", "mixtral", 2, 256, 4, 1024, n_positions=256, ffn_dim=256,
                                n_kv_head=2, n_experts=4, top_k=2, tie_embeddings=False),
}
# one full-width layer of the big models (every kernel shape of the real model, S = 512):
# GPU numerics tests against the fp32 reference
PRESETS["llama3-8b-1l"] = PRESETS["llama3-8b"].with_(name="llama3-8b-1l", n_layer=1)
PRESETS["mixtral-8x7b-1l"] = PRESETS["mixtral-8x7b"].with_(name="mixtral-8x7b-1l", n_layer=1)
PRESETS["gpt2-small"] = PRESETS["gpt2"].with_(name="gpt2-small")
PRESETS["llama-3-8b"] = PRESETS["llama3-8b"]
PRESETS["mixtral"] = PRESETS["mixtral-8x7b"]


def get_config(name: str) -> ModelConfig:
    try:
        return PRESETS[name]
    except KeyError:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}") from None
