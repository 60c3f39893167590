#!/usr/bin/env python3
"""Grouped MoE-expert GEMM probe: every candidate config of ``ops.gemm_grouped`` for a shape
(8 experts x M routed rows, cold weights), with the achieved weight-stream bandwidth.

    python benchmarks/bench_grouped.py M,N,K[,s] ...      (s = SwiGLU gate/up launch)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402


def main():
    ext = ops.ext()
    for spec in sys.argv[1:]:
        parts = spec.split(",")
        M, N, K = (int(v) for v in parts[:3])
        sw = len(parts) > 3 and "s" in parts[3]
        best, res = tuning._tune_grouped(ext, M, N, K, torch.device("cuda"), 4 if sw else 0,
                                         ("s" if sw else "") + "g", save=False)
        wbytes = tuning.GROUPS * N * K * 2
        rows = sorted(((round(t, 1), c) for (c, _), t in res.items()))
        print(json.dumps({"M": M, "N": N, "K": K, "swiglu": sw, "best": best[:2], "best_us": round(best[2], 1),
                          "best_TBps": round(wbytes / best[2] / 1e6, 2), "all_us": rows}), flush=True)


if __name__ == "__main__":
    main()
