#!/usr/bin/env python3
"""Cost of the DAG's fused GEMM epilogues on GPT-2's shapes: plain GEMM vs the same GEMM
with a folded LayerNorm (statistics handed over by the producer), bias, GeLU, residual and
row-statistics output, at the tuned config, hot and cold weights. hipGraph-timed.

    python benchmarks/bench_fused_epilogue.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402
from distributed_llm_scheduler_amd.ops.tuning import _graph_time  # noqa: E402


def main():
    dev = "cuda"
    for (M, N, K, act) in ((512, 2304, 768, None), (512, 3072, 768, "gelu"), (512, 768, 768, None),
                           (512, 768, 3072, None)):
        x = torch.randn(M, K, device=dev).bfloat16()
        ncopy = max(1, (400 << 20) // (N * K * 2))
        ws = [(torch.randn(N, K, device=dev) * 0.05).bfloat16() for _ in range(ncopy)]
        nw = torch.ones(K, device=dev).bfloat16()
        nb = torch.zeros(K, device=dev).bfloat16()
        bias = torch.zeros(N, device=dev).bfloat16()
        derived = [ops.derive_norm_gemm(w, nw, nb, bias) for w in ws[:1]]
        wd, cs, bd = derived[0]
        stats = torch.zeros(M, 2, device=dev)
        stats[:, 1] = K
        res = torch.randn(M, N, device=dev).bfloat16()
        sout = torch.zeros(M, 2, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cfg = tuning.lookup_fused(M, N, K)
        row = {"M": M, "N": N, "K": K, "cfg": cfg}
        row["plain_hot"] = round(_graph_time(lambda i: ops.linear(x, ws[0], out=out), reps=20), 2)
        row["plain_cold"] = round(_graph_time(lambda i: ops.linear(x, ws[i % ncopy], out=out), reps=ncopy), 2)
        if K <= 1024:
            row["ln_fold_ext_stats"] = round(_graph_time(
                lambda i: ops.linear_norm(x, wd, cs, bd, "layernorm", act=act, out=out, ext_stats=stats), reps=20), 2)
            row["ln_fold_inkernel"] = round(_graph_time(
                lambda i: ops.linear_norm(x, wd, cs, bd, "layernorm", act=act, out=out), reps=20), 2)
        row["bias_res_stats"] = round(_graph_time(
            lambda i: ops.linear(x, ws[0], bias=bias, residual=res, out=out, stats_out=sout), reps=20), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
