#!/usr/bin/env python3
"""GEMM time vs K at fixed (M, N): the intercept is the per-kernel fixed cost (launch,
prologue, epilogue), the slope the per-K-tile main-loop cost. Hot weights, hipGraph-timed.

    python benchmarks/bench_gemm_ksweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops.tuning import _graph_time  # noqa: E402


def main():
    ext = ops.ext()
    for M, N in ((512, 768), (512, 3072), (512, 50304)):
        for cfg in ((0, 8) if N > 4096 else (3,)):
            row = {"M": M, "N": N, "cfg": cfg}
            for K in (64, 128, 256, 512, 768, 1536, 3072):
                x = torch.randn(M, K, device="cuda").bfloat16()
                w = torch.randn(N, K, device="cuda").bfloat16()
                o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                row[K] = round(_graph_time(lambda i: ext.gemm(x, w, None, None, 0, 1.0, o, cfg, 1), reps=20), 2)
            print(json.dumps(row), flush=True)
        row = {"M": M, "N": N, "cfg": "torch"}
        for K in (64, 768, 3072):
            x = torch.randn(M, K, device="cuda").bfloat16()
            w = torch.randn(N, K, device="cuda").bfloat16()
            o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row[K] = round(_graph_time(lambda i: torch.matmul(x, w.t(), out=o), reps=20), 2)
        row["fill"] = round(_graph_time(lambda i: o.fill_(1.0), reps=20), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
