#!/usr/bin/env python3
"""Per-kernel fixed cost on MI355X inside a hipGraph, and hot- vs cold-weight GEMM time.

Answers "how much of a DAG step is kernel-boundary overhead?": a graph of R back-to-back
launches of a trivial kernel gives the per-launch floor (dispatch + end-of-kernel L2
writeback across the 8 XCDs); the GPT-2 GEMMs are then timed with hot weights (one copy,
L2/MALL resident) and cold weights (a ring of copies larger than the 256 MiB MALL).

    python benchmarks/bench_launch_floor.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops.tuning import _graph_time  # noqa: E402


def main():
    ext = ops.ext()
    dev = "cuda"
    for n in (64, 512 * 768, 512 * 3072):
        a = torch.randn(n, device=dev).bfloat16()
        b = torch.randn(n, device=dev).bfloat16()
        o = torch.empty_like(a)
        t = _graph_time(lambda i: ext.add(a, b, out=o), reps=100, rounds=5)
        print(json.dumps({"case": "add", "elems": n, "us": round(t, 3)}), flush=True)
    x = torch.randn(512, 768, device=dev).bfloat16()
    w = torch.ones(768, device=dev).bfloat16()
    bb = torch.zeros(768, device=dev).bfloat16()
    y = torch.empty_like(x)
    t = _graph_time(lambda i: ext.norm(x, w, bb, 1e-5, out=y), reps=100, rounds=5)
    print(json.dumps({"case": "layernorm", "shape": [512, 768], "us": round(t, 3)}), flush=True)
    for (M, N, K) in ((512, 2304, 768), (512, 768, 768), (512, 3072, 768), (512, 768, 3072), (512, 50257, 768)):
        xa = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
        ncopy = max(1, min(64, int(400e6 // (N * K * 2)) + 1))
        ws = [(torch.randn(N, K, device=dev) * 0.05).bfloat16() for _ in range(ncopy)]
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        row = {"case": "gemm", "M": M, "N": N, "K": K, "cold_copies": ncopy}
        for cfg, sk in ((-1, 0),) + tuple((c, s) for c in (3, 5, 2, 1, 4) for s in (1, 2, 4)):
            if K % (64 * max(sk, 1)):
                continue
            try:
                hot = _graph_time(lambda i: ext.gemm(xa, ws[0], None, None, 0, 1.0, out, cfg, sk), reps=20, rounds=5)
                cold = _graph_time(lambda i: ext.gemm(xa, ws[i % ncopy], None, None, 0, 1.0, out, cfg, sk),
                                   reps=ncopy if ncopy > 1 else 20, rounds=5)
            except RuntimeError as e:  # config not valid for this shape
                row[f"c{cfg}s{sk}"] = str(e)[:40]
                continue
            row[f"c{cfg}s{sk}"] = [round(hot, 2), round(cold, 2), round(flops / cold / 1e6, 1)]
        tm = _graph_time(lambda i: torch.matmul(xa, ws[i % ncopy].t(), out=out), reps=ncopy if ncopy > 1 else 20,
                         rounds=5)
        row["torch_cold"] = round(tm, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
