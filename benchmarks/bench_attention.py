#!/usr/bin/env python3
"""Attention variants (csrc/kernels/attention.hip launch_variant) timed in a hipGraph for the
DAG shapes: GPT-2 (12 heads, D=64), Llama-3-8B / Mixtral (32 q / 8 kv heads, D=128), S=512,
causal, batch 1. One JSON line per shape: microseconds per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402

SHAPES = [("gpt2", 1, 512, 12, 12, 64), ("llama", 1, 512, 32, 8, 128)]


def main():
    e = ops.ext()
    nvar = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    for name, B, S, nh, nkv, D in SHAPES:
        qkv = (torch.randn(B * S, (nh + 2 * nkv) * D, device="cuda") * 0.5).bfloat16()
        q, k, v = qkv[:, :nh * D], qkv[:, nh * D:(nh + nkv) * D], qkv[:, (nh + nkv) * D:]
        o = torch.empty(B * S, nh * D, device="cuda", dtype=torch.bfloat16)
        row = {"shape": name}
        for var in range(nvar):
            fn = lambda i, var=var: e.attention(q, k, v, B, S, nh, nkv, D, True, D ** -0.5, o, var, 0, 0)  # noqa: E731
            row[var] = round(tuning._graph_time(fn, reps=20, rounds=5), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
