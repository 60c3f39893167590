#!/usr/bin/env python3
"""Would two concurrent half-size chains fill the launch gaps of the GPT-2 step? The 48 layer
GEMMs of GPT-2 (12 x QKV / out-proj / fc1 / fc2) in one hipGraph as (a) one chain at M = 512
(the DAG today), (b) two M = 256 chains (the request split into two sequence chunks) forked on
two streams inside the graph, (c) the same two chains on one stream. Tuned configs per shape.

    python benchmarks/bench_two_chains.py
"""
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
    torch.cuda.synchronize()
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
    e = ops.ext()
    H, F = 768, 3072
    shapes = [(3 * H, H), (H, H), (F, H), (H, F)]
    tuning.ensure_tuned([(m, n, k) for m in (256, 512) for n, k in shapes], "cuda")
    torch.manual_seed(0)
    layers = [[(torch.randn(n, k, device="cuda") * 0.05).bfloat16() for n, k in shapes] for _ in range(12)]

    def bufs(M):
        x = (torch.randn(M, H, device="cuda") * 0.5).bfloat16()
        xf = (torch.randn(M, F, device="cuda") * 0.5).bfloat16()
        outs = [torch.empty(M, n, device="cuda", dtype=torch.bfloat16) for n, _ in shapes]
        cfgs = [tuning.lookup(M, n, k) for n, k in shapes]
        return x, xf, outs, cfgs

    b512, b256a, b256b = bufs(512), bufs(256), bufs(256)

    def chain(b):
        x, xf, outs, cfgs = b
        for ws in layers:
            for (c, k), a, w, o in zip(cfgs, (x, x, x, xf), ws, outs):
                e.gemm(a, w, None, None, 0, 1.0, o, c, k, stream_pol=4)

    side = torch.cuda.Stream()

    def two_streams():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        chain(b256a)
        with torch.cuda.stream(side):
            chain(b256b)
        cur.wait_stream(side)

    res = {"cfgs_512": b512[3], "cfgs_256": b256a[3],
           "one_chain_512_us": round(graph_us(lambda: chain(b512)), 1),
           "two_chains_256_two_streams_us": round(graph_us(two_streams), 1),
           "two_chains_256_one_stream_us": round(graph_us(lambda: (chain(b256a), chain(b256b))), 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
