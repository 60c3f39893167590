#!/usr/bin/env python3
"""Shape probe: our GEMM configs vs torch.matmul at given (M, N, K), hot operands,
hipGraph-timed. ``python benchmarks/bench_gemm_shapes.py M,N,K[,cfgs] ...``"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops.tuning import _graph_time  # noqa: E402


def main():
    ext = ops.ext()
    for spec in sys.argv[1:]:
        parts = spec.split(",")
        M, N, K = (int(v) for v in parts[:3])
        cfgs = [int(c) for c in parts[3].split("/")] if len(parts) > 3 else [0, 3]
        sk = int(parts[4]) if len(parts) > 4 else 1
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        row = {"M": M, "N": N, "K": K, "splitk": sk}
        for c in cfgs:
            row[f"c{c}"] = round(_graph_time(lambda i: ext.gemm(x, w, None, None, 0, 1.0, o, c, sk), reps=20), 2)
        row["torch"] = round(_graph_time(lambda i: torch.matmul(x, w.t(), out=o), reps=20), 2)
        row["fill"] = round(_graph_time(lambda i: o.fill_(1.0), reps=20), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
