#!/usr/bin/env python3
"""Does the total weight footprint change per-GEMM speed? Times the MoE expert gate_up GEMM
(ranged rows, SwiGLU epilogue) cycling over `n` distinct weights carved from one slab, for
several n (4 -> 940 MB ... 256 -> 60 GB), and the same for a plain dense GEMM."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402


def main():
    e = ops.ext()
    N, K, R = 28672, 4096, 1024
    x = (torch.randn(R, K, device="cuda") * 0.5).bfloat16()
    out = torch.empty(R, N // 2, device="cuda", dtype=torch.bfloat16)
    rows = torch.tensor([300, 428], dtype=torch.int32, device="cuda")
    per = N * K * 2
    for n in (4, 16, 64, 256):
        slab = torch.empty(n * per, dtype=torch.uint8, device="cuda")
        ws = [slab[i * per:(i + 1) * per].view(torch.bfloat16).view(N, K) for i in range(n)]
        for w in ws:
            w.normal_(0, 0.02)
        for cfg, sk in ((9, 1), (7, 1), (0, 1)):
            t = tuning._graph_time(lambda i: e.gemm(x, ws[i % n], None, None, 4, 1.0, out, cfg, sk, None, 0, 1e-5,
                                                    rows), reps=n, rounds=3)
            print(json.dumps({"n_weights": n, "footprint_gb": round(n * per / 1e9, 1), "cfg": cfg, "us": round(t, 1),
                              "w_TBs": round(per / t / 1e6, 2)}), flush=True)
        del ws, slab
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
