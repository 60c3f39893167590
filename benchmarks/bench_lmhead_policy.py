#!/usr/bin/env python3
"""Cache policy of the GPT-2 LM head (GemmArgs::stream_pol): does streaming its 77 MB weight
(nt DMA) and / or its 51 MB of logits (nt stores) keep the 170 MB of layer weights resident in
the 256 MB Infinity Cache across steps? A synthetic GPT-2 step in one hipGraph: 12 x the four
layer GEMMs with their tuned configs, then the LM head exactly as the DAG issues it (folded
final LayerNorm, handed-over row statistics, logits rows padded to 50304); per policy the
step, the layers alone inside the step's cache state, and the LM head alone.

    python benchmarks/bench_lmhead_policy.py [--pols 0,1,2,3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402


def graph_us(fn, reps=30):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pols", default="0,1,2,3")
    args = ap.parse_args()
    e = ops.ext()
    M, H, F, V, VP = 512, 768, 3072, 50257, 50304
    torch.manual_seed(0)
    shapes = [(3 * H, H), (H, H), (F, H), (H, F)]
    layers = [[(torch.randn(n, k, device="cuda") * 0.05).bfloat16() for n, k in shapes] for _ in range(12)]
    cfgs = [tuning.lookup(M, n, k) for n, k in shapes]
    x = (torch.randn(M, H, device="cuda") * 0.5).bfloat16()
    xf = (torch.randn(M, F, device="cuda") * 0.5).bfloat16()
    outs = [torch.empty(M, n, device="cuda", dtype=torch.bfloat16) for n, _ in shapes]
    wte = (torch.randn(V, H, device="cuda") * 0.05).bfloat16()
    cs = wte.float().sum(1).contiguous()
    st = torch.stack([x.float().sum(1), (x.float() ** 2).sum(1)], 1).contiguous()
    lb = torch.empty(M, VP, device="cuda", dtype=torch.bfloat16)
    logits = lb[:, :V]
    cfg, sk = tuning.lookup_fused(M, V, H)

    def layers_only():
        for ws in layers:
            for (c, k), a, w, o in zip(cfgs, (x, x, x, xf), ws, outs):
                e.gemm(a, w, None, None, 0, 1.0, o, c, k)

    res = {"lmhead_cfg": [cfg, sk]}
    for pol in (int(p) for p in args.pols.split(",")):
        def head():
            e.gemm(x, wte, None, None, 0, 1.0, logits, cfg, sk, cs, 1, 1e-5, None, False, None, None, 1, 2, 0, None,
                   st, stream_pol=pol)

        def step():
            layers_only()
            head()

        res[f"pol{pol}_step_us"] = round(graph_us(step), 1)
        res[f"pol{pol}_lmhead_alone_us"] = round(graph_us(head), 1)
    res["layers_alone_us"] = round(graph_us(layers_only), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
