#!/usr/bin/env python3
"""Shape probe: our GEMM configs vs torch.matmul at given (M, N, K), hipGraph-timed.

    python benchmarks/bench_gemm_shapes.py M,N,K[,cfg/cfg/...[,splitk[,flags]]] ...

flags (any of): ``r`` = MoE-expert launch (M routed rows at a device-side row range inside a
4*M-row activation), ``s`` = SwiGLU epilogue (N interleaved gate/up rows -> N/2 outputs),
``c`` = cold weights (a ring of weight copies larger than the 256 MiB Infinity Cache).
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
    for spec in sys.argv[1:]:
        parts = spec.split(",")
        M, N, K = (int(v) for v in parts[:3])
        cfgs = [int(c) for c in parts[3].split("/")] if len(parts) > 3 else [0, 3]
        sk = int(parts[4]) if len(parts) > 4 else 1
        flags = parts[5] if len(parts) > 5 else ""
        ranged, sw, cold = "r" in flags, "s" in flags, "c" in flags
        rows_total = 4 * M if ranged else M
        x = torch.randn(rows_total, K, device="cuda").bfloat16()
        ncopy = max(1, min(32, (512 << 20) // (N * K * 2) + 1)) if cold else 1
        ws = [torch.randn(N, K, device="cuda").bfloat16() for _ in range(ncopy)]
        o = torch.empty(rows_total, N // 2 if sw else N, device="cuda", dtype=torch.bfloat16)
        rng = torch.tensor([M, 2 * M], dtype=torch.int32, device="cuda") if ranged else None
        act = 4 if sw else 0
        row = {"M": M, "N": N, "K": K, "splitk": sk, "flags": flags, "weight_copies": ncopy}
        reps = max(ncopy, 20)
        for c in cfgs:
            try:
                row[f"c{c}"] = round(_graph_time(
                    lambda i: ext.gemm(x, ws[i % ncopy], None, None, act, 1.0, o, c, sk, None, 0, 1e-5, rng),
                    reps=reps), 2)
            except RuntimeError as e:
                row[f"c{c}"] = str(e)[:60]
        if not (ranged or sw):
            row["torch"] = round(_graph_time(lambda i: torch.matmul(x, ws[i % ncopy].t(), out=o), reps=reps), 2)
        wbytes = N * K * 2
        row["weight_GBps_best"] = round(wbytes / min(v for k, v in row.items()
                                                     if k.startswith("c") and isinstance(v, float)) / 1e3, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
