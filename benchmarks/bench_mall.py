#!/usr/bin/env python3
"""How much do the GPT-2 layer GEMMs gain when their weights hit in the Infinity Cache (MALL)
instead of streaming from HBM? Each shape runs with its tuned config in a hipGraph that
rotates over enough weight copies to make the weight footprint F MB: F = one copy is hot in
L2/MALL, F above the 256 MB MALL streams from HBM every call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402

SHAPES = [("qkv", 512, 2304, 768), ("out", 512, 768, 768), ("fc1", 512, 3072, 768), ("fc2", 512, 768, 3072)]


def main():
    e = ops.ext()
    for name, M, N, K in SHAPES:
        cfg, sk = tuning.lookup(M, N, K)
        x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        wbytes = N * K * 2
        row = {"shape": name, "cfg": [cfg, sk]}
        for mb in (0, 96, 160, 224, 384, 768):
            copies = max(1, (mb << 20) // wbytes)
            ws = [(torch.randn(N, K, device="cuda") * 0.05).bfloat16() for _ in range(copies)]
            if cfg >= tuning.REGSTAGE or cfg == tuning.LIB:
                fn = lambda i: torch.mm(x, ws[i % copies].t(), out=out)  # noqa: E731
            else:
                fn = lambda i: e.gemm(x, ws[i % copies], None, None, 0, 1.0, out, cfg, sk)  # noqa: E731
            reps = max(copies, 20)
            row[f"{copies * wbytes >> 20}MB_us"] = round(tuning._graph_time(fn, reps=reps, rounds=3), 2)
            del ws
            torch.cuda.empty_cache()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
