#!/usr/bin/env python3
"""GPT-2 LM head as the DAG issues it (512 x 50257 x 768, folded final LayerNorm with handed-over
row statistics, logits into rows padded to 50304), hipGraph-timed with cold weights: the single
tuned launch (1.54 rounds of 256 x 256 tiles) against the column split of ops/gemm_tuning.json
(a whole round of 256 x 256 tiles + one round of 256 x 144 tiles), and any other split given.

    python benchmarks/bench_lmhead_split.py [--at 32768] [--tail-cfg 42]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402
from distributed_llm_scheduler_amd.ops.tuning import _graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--at", default="32768")
    ap.add_argument("--tail-cfg", default="42")
    a = ap.parse_args()
    M, N, K = 512, 50257, 768
    torch.manual_seed(0)
    x = (torch.randn(1, M, K, device="cuda") * 2).bfloat16()
    ws = [(torch.randn(N, K, device="cuda") * 0.05).bfloat16() for _ in range(4)]  # 4 x 77 MB: MALL-cold
    cs = ws[0].float().sum(1).contiguous()
    xf = x.view(M, K).float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).contiguous()
    ob = torch.empty(1, M, 50304, device="cuda", dtype=torch.bfloat16)
    out = ob[:, :, :N]
    key = tuning._key(M, N, K)
    tuning.table()
    saved = tuning._col_splits.get(key)
    base_cfg = tuning.lookup_fused(M, N, K)

    def run(i):
        ops.linear_norm(x, ws[i % 4], cs, None, "layernorm", out=out, ext_stats=st)

    res = []
    tuning._col_splits.pop(key, None)
    res.append({"variant": f"single launch cfg {base_cfg}", "us": round(_graph_time(run, reps=8), 2)})
    for at in (int(v) for v in a.at.split(",")):
        for tc in (int(v) for v in a.tail_cfg.split(",")):
            tuning._col_splits[key] = [(0, at, base_cfg[0], 1), (at, N, tc, 1)]
            res.append({"variant": f"split at {at}: cfg {base_cfg[0]} + tail cfg {tc}",
                        "us": round(_graph_time(run, reps=8), 2)})
    if saved is not None:
        tuning._col_splits[key] = saved
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
