#!/usr/bin/env python3
"""Cold-weight GEMM landscape: every config of our LDS-DMA kernel (and split-K) vs
torch.matmul (hipBLASLt) with weights rotated through > 512 MiB of copies, so each call
streams its weight from HBM as a once-per-step DAG layer does. One JSON line per shape.

    python benchmarks/bench_cold_gemm.py [--shapes llama|mixtral|gpt2|all]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402

SHAPES = {
    "gpt2": [(512, 2304, 768), (512, 768, 768), (512, 3072, 768), (512, 768, 3072), (512, 50257, 768)],
    "llama": [(512, 6144, 4096), (512, 4096, 4096), (512, 28672, 4096), (512, 4096, 14336), (512, 128256, 4096)],
    "mixtral": [(128, 28672, 4096), (128, 4096, 14336), (256, 28672, 4096), (256, 4096, 14336)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    shapes = sum(SHAPES.values(), []) if a.shapes == "all" else SHAPES[a.shapes]
    e = ops.ext()
    for M, N, K in shapes:
        x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        wbytes = N * K * 2
        copies = max(2, min(64, (768 << 20) // wbytes + 1))
        ws = [(torch.randn(N, K, device="cuda") * 0.05).bfloat16() for _ in range(copies)]
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {}
        res["torch"] = tuning._graph_time(lambda i: torch.matmul(x, ws[i % copies].t(), out=out), reps=copies)
        for cfg, sk in tuning.candidates(M, N, K, e.gemm_glds_num_configs()):
            try:
                res[f"c{cfg}s{sk}"] = tuning._graph_time(
                    lambda i: e.gemm(x, ws[i % copies], None, None, 0, 1.0, out, cfg, sk), reps=copies)
            except RuntimeError:
                pass
        best = sorted(res.items(), key=lambda kv: kv[1])[:a.top]
        fl = 2.0 * M * N * K
        row = {"M": M, "N": N, "K": K, "copies": copies, "torch_us": round(res["torch"], 1),
               "torch_tf": round(fl / res["torch"] / 1e6), "torch_wTBs": round(wbytes / res["torch"] / 1e6, 2),
               "best": [(k, round(v, 1), round(fl / v / 1e6)) for k, v in best],
               "best_wTBs": round(wbytes / best[0][1] / 1e6, 2)}
        print(json.dumps(row), flush=True)
        del ws


if __name__ == "__main__":
    main()
