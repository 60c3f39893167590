#!/usr/bin/env python3
"""Do independent branches of a captured hipGraph run concurrently on MI355X? A host-pull
refill (32 workgroups, ~0.7 ms for 38 MB) forked onto a side stream beside a chain of GEMMs
on the main stream: eager streams vs the same work captured in one hipGraph."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ext = ops.ext()
    n = 38 << 20
    src = torch.randint(0, 255, (n,), dtype=torch.uint8).pin_memory()
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    x = torch.randn(512, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(768, 768, device="cuda", dtype=torch.bfloat16)
    side = torch.cuda.Stream()

    def gemms():
        y = x
        for _ in range(60):
            y = torch.mm(y, w)
        return y

    def pull():
        ext.host_pull(dst, src, 32)

    def both():
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            pull()
        gemms()
        torch.cuda.current_stream().wait_stream(side)

    res = {"gemms_ms": timed(gemms), "pull_ms": timed(pull), "both_eager_ms": timed(both)}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        both()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        both()
    res["both_graph_ms"] = timed(g.replay)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        gemms()
    res["gemms_graph_ms"] = timed(g2.replay)
    print(json.dumps({k: round(v, 4) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
